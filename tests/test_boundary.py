"""C-ABI boundary checks that need no GPU: the library loads, exports every function
include/wk_api.h declares, and rejects unsupported configurations before touching a
device (Hyperparameters validation, Hyperparameters.cs:189-217)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "wk_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(wk_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_lists_functions():
    fns = header_functions()
    assert "wk_create" in fns and "wk_ppo_update" in fns and len(fns) >= 30


def test_library_exports_every_symbol(wk):
    lib = wk.load_library()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(wk.EXPORTS) == header_functions()


def test_struct_layouts(wk):
    assert C.sizeof(wk.PairTrace) == 388
    assert C.sizeof(wk.BodyView) == 4 + 48 + 8 + 8 + 4 + 4 + 4 + 4
    lib = wk.load_library()
    cfg = wk.default_config()
    assert cfg.Iterations == 50 and cfg.MaxTimesteps == 1000 and cfg.Epochs == 5
    assert cfg.BatchSize == 64 and cfg.UseGAE == 0 and cfg.NormalizeAdvantages == 0
    assert abs(cfg.Gamma - 0.9) < 1e-7 and abs(cfg.Lambda - 0.95) < 1e-7
    assert abs(cfg.Epsilon - 0.3) < 1e-7 and cfg.LogStandardDeviation == -1.0
    assert abs(cfg.Alpha - 1e-3) < 1e-10 and abs(cfg.AdamEpsilon - 1e-8) < 1e-15
    assert cfg.DeltaTime == C.c_float(166667 / 1e7).value
    assert lib.wk_version().decode().startswith("wk")


@pytest.mark.parametrize("field,value,msg", [
    ("Iterations", 0, "iterations"),
    ("Iterations", 200, "iterations"),
    ("Epochs", 50, "epochs"),
    ("BatchSize", 0, "batch size"),
    ("Gamma", 1.5, "gamma"),
    ("Epsilon", 0.0, "epsilon"),
    ("LogStandardDeviation", 5.0, "log standard deviation"),
    ("GameSpeed", 10, "game speed"),
    ("ActorNeuralNetwork", "Input |32| (ReLU) |4| Output", "actor network"),
])
def test_invalid_config_rejected_without_gpu(wk, field, value, msg):
    lib = wk.load_library()
    cfg = wk.default_config(**{field: value})
    h = C.c_void_p()
    rc = lib.wk_create(C.byref(cfg), 0, 8, 1, C.byref(h))
    assert rc == -3  # WK_ERR_CONFIG
    assert msg.lower() in lib.wk_last_error(None).decode().lower()
    assert not h.value


def test_default_network_strings_accepted(wk):
    cfg = wk.default_config(CriticNeuralNetwork="Input |64| (LeakyReLU) |1| Output",
                            ActorNeuralNetwork="Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output")
    lib = wk.load_library()
    h = C.c_void_p()
    rc = lib.wk_create(C.byref(cfg), 0, 8, 1, C.byref(h))
    # on a GPU box this succeeds; without a device it fails loudly with a HIP error
    assert rc in (0, -2)
    if rc == 0:
        lib.wk_destroy(h)
    else:
        assert "device" in lib.wk_last_error(None).decode().lower()


def test_bad_arguments(wk):
    lib = wk.load_library()
    h = C.c_void_p()
    assert lib.wk_create(None, 0, 0, 1, C.byref(h)) == -1
    assert lib.wk_destroy(None) == 0
    assert lib.wk_step(None, None, 1, None, None, None, None) == -1


def test_rough_floor_accepted_on_every_mapping(wk):
    """RoughFloor runs on every mapping (1, 2, 4 and 16 lanes per walker, and auto): the
    configuration is never refused (without a GPU the create fails later, at the device)"""
    lib = wk.load_library()
    for lanes in (0, 1, 2, 4, 16):
        cfg = wk.default_config(RoughFloor=1, LanesPerWalker=lanes)
        h = C.c_void_p()
        rc = lib.wk_create(C.byref(cfg), 0, 4, 1, C.byref(h))
        if rc == 0:
            lib.wk_destroy(h)
        assert rc != -3, (lanes, lib.wk_last_error(None))