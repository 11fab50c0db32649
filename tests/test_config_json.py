"""JSON configuration files, through the C ABI with no GPU.

Reference: Hyperparameters.SerializeJson / DeserializeJson (Hyperparameters.cs:124-187)
over SerializableHyperparameters (:11-77) with System.Text.Json defaults,
ValidateHyperparameterValues (:189-217) and ValidateVariables (:240-290, validators in
ConsoleRenderer.cs:639-682).  The reference ships no configuration files, so the text is
pinned by System.Text.Json's documented defaults (declaration-order properties, two-space
indentation, shortest round-trip floats, JavaScriptEncoder.Default escaping) -- "parity
unpinned" against a real .NET run.
"""
import ctypes as C
import os

import numpy as np
import pytest

CRITIC = "Input |64| (LeakyReLU) |1| Output"
ACTOR = "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output"
INT_FIELDS = ["GameSpeed", "Iterations", "MaxTimesteps", "Epochs", "BatchSize"]
BOOL_CFG = ["RoughFloor", "UseGAE", "NormalizeAdvantages"]
FLOAT_FIELDS = ["Alpha", "Beta1", "Beta2", "AdamEpsilon", "Gamma", "Lambda", "Epsilon",
                "LogStandardDeviation"]


def expected_default_text(file_path):
    return "\n".join([
        "{",
        '  "GameSpeed": 1,',
        '  "CollectData": true,',
        '  "SaveWeights": true,',
        '  "Iterations": 50,',
        '  "MaxTimesteps": 1000,',
        '  "RoughFloor": false,',
        f'  "CriticNeuralNetwork": "{CRITIC}",',
        f'  "ActorNeuralNetwork": "{ACTOR}",',
        '  "CriticWeightFileName": "critic",',
        '  "ActorWeightFileName": "actor",',
        f'  "FilePath": "{file_path}",',
        '  "Alpha": 0.001,',
        '  "Beta1": 0.9,',
        '  "Beta2": 0.999,',
        '  "AdamEpsilon": 1E-08,',
        '  "Epochs": 5,',
        '  "BatchSize": 64,',
        '  "UseGAE": false,',
        '  "NormalizeAdvantages": false,',
        '  "Gamma": 0.9,',
        '  "Lambda": 0.95,',
        '  "Epsilon": 0.3,',
        '  "LogStandardDeviation": -1',
        "}",
    ])


def snapshot(cfg, host):
    d = {f: getattr(cfg, f) for f, _ in type(cfg)._fields_ if "NeuralNetwork" not in f}
    d.update({f: getattr(host, f) for f, _ in type(host)._fields_})
    return d


def test_default_document(wk):
    host = wk.default_host_settings()
    assert host.FilePath.endswith(b"/") and os.path.isdir(host.FilePath.decode())
    assert wk.config_to_json() == expected_default_text(host.FilePath.decode())


def test_round_trip_random_values(wk, tmp_path):
    rng = np.random.default_rng(11)
    for _ in range(50):
        cfg = wk.default_config()
        for f, (lo, hi) in dict(GameSpeed=(1, 9), Iterations=(1, 199), MaxTimesteps=(1, 10**6),
                                Epochs=(1, 49), BatchSize=(1, 999)).items():
            setattr(cfg, f, int(rng.integers(lo, hi + 1)))
        for f in BOOL_CFG:
            setattr(cfg, f, int(rng.integers(0, 2)))
        cfg.Alpha = np.float32(rng.uniform(1e-9, 9.9))
        for f in ["Beta1", "Beta2", "Gamma", "Lambda", "Epsilon"]:
            setattr(cfg, f, np.float32(rng.uniform(1e-7, 1.0)))
        cfg.AdamEpsilon = np.float32(10 ** rng.uniform(-30, -0.01))
        cfg.LogStandardDeviation = np.float32(rng.uniform(-4.99, 4.99))
        host = wk.default_host_settings()
        host.CollectData, host.SaveWeights = int(rng.integers(0, 2)), int(rng.integers(0, 2))
        host.FilePath = (str(tmp_path) + "/").encode()
        text = wk.config_to_json(cfg, host)
        cfg2, host2, fixes = wk.config_from_json(text)
        assert fixes == []
        for f in INT_FIELDS + BOOL_CFG:
            assert getattr(cfg2, f) == getattr(cfg, f), f
        for f in FLOAT_FIELDS:  # bit-exact through the shortest round-trip digits
            assert np.float32(getattr(cfg2, f)).view(np.uint32) == \
                np.float32(getattr(cfg, f)).view(np.uint32), f
        assert snapshot(wk.default_config(), host2)["FilePath"] == host.FilePath
        assert (host2.CollectData, host2.SaveWeights) == (host.CollectData, host.SaveWeights)
        assert cfg2.CriticNeuralNetwork == CRITIC.encode() and cfg2.ActorNeuralNetwork == ACTOR.encode()


def test_missing_unknown_duplicate_and_case(wk):
    base = wk.default_config(Epochs=7, Gamma=0.5)
    cfg, _, _ = wk.config_from_json(
        '{"Epochs": 3, "epochs": 40, "Unknown": {"x": [1, 2, {"y": null}]}, "Epochs": 4}', base)
    assert cfg.Epochs == 4  # last duplicate wins, other casing ignored
    assert cfg.Gamma == np.float32(0.5) and cfg.Iterations == 50  # missing keep their value


def test_null_document_changes_nothing(wk):
    base = wk.default_config(Epochs=7)
    cfg, _, fixes = wk.config_from_json("null", base)
    assert cfg.Epochs == 7 and fixes == []


@pytest.mark.parametrize("doc", [
    '{"Epochs": 1.0}', '{"Epochs": "5"}', '{"Epochs": null}', '{"Epochs": 1e1}',
    '{"Epochs": 99999999999}', '{"Alpha": true}', '{"Alpha": 1e39}', '{"Alpha": "0.1"}',
    '{"UseGAE": 1}', '{"UseGAE": "true"}', '{"FilePath": 5}', '{"Epochs": 5,}',
    '{"Epochs": 5 // c\n}', "[1]", '"text"', '{"Epochs": 5} x', "", "{", '{"A": tru}',
    '{"A": 01}', '{"A": "\\x"}', '{"A": "\\ud800"}',
])
def test_malformed_documents_rejected(wk, doc):
    base = wk.default_config(Epochs=7)
    before = snapshot(base, wk.default_host_settings())
    with pytest.raises(wk.WkError, match="JSON deserializer error"):
        wk.config_from_json(doc, base)
    assert snapshot(base, wk.default_host_settings()) == before


@pytest.mark.parametrize("field,bad,good", [
    ("GameSpeed", [0, 10], [1, 9]), ("Iterations", [0, 200], [1, 199]),
    ("MaxTimesteps", [0, -1], [1, 10**9]), ("Epochs", [0, 50], [1, 49]),
    ("BatchSize", [0, 1000], [1, 999]), ("Alpha", [0, 10, -1], [1e-30, 9.99]),
    ("Beta1", [0, 1.01], [1e-6, 1]), ("Beta2", [0, 1.5], [1e-6, 1]),
    ("AdamEpsilon", [0, 1], [1e-30, 0.99]), ("Gamma", [0, 1.01], [1e-6, 1]),
    ("Lambda", [0, 2], [0.5, 1]), ("Epsilon", [0, 1.1], [0.01, 1]),
    ("LogStandardDeviation", [-5, 5], [-4.99, 4.99]),
])
def test_value_ranges(wk, field, bad, good):
    """ValidateHyperparameterValues (Hyperparameters.cs:189-217): open / half-open ranges"""
    for v in bad:
        base = wk.default_config()
        with pytest.raises(wk.WkError, match="Invalid"):
            wk.config_from_json('{"%s": %s}' % (field, v), base)
        assert getattr(base, field) == getattr(wk.default_config(), field)
    for v in good:
        cfg, _, _ = wk.config_from_json('{"%s": %s}' % (field, v))
        assert getattr(cfg, field) == pytest.approx(v, rel=1e-7)


def test_validate_variables_resets(wk, tmp_path):
    """ValidateVariables (Hyperparameters.cs:240-290): bad path / names / networks revert"""
    good_dir = str(tmp_path) + "/"
    cfg, host, fixes = wk.config_from_json(
        '{"FilePath": "%s", "CriticWeightFileName": "my critic", "ActorWeightFileName": "a+b"}'
        % good_dir)
    assert fixes == [] and host.FilePath == good_dir.encode()
    assert host.CriticWeightFileName == b"my critic" and host.ActorWeightFileName == b"a+b"
    cfg, host, fixes = wk.config_from_json(
        '{"Epochs": 9, "FilePath": "%s", "CriticWeightFileName": "x/y", "ActorWeightFileName": null,'
        ' "CriticNeuralNetwork": "Input |64| (Sigmoid) |1| Output",'
        ' "ActorNeuralNetwork": "Input |64| (TanH) |2| Output"}' % str(tmp_path))
    assert cfg.Epochs == 9  # applied before the variables are checked
    assert host.FilePath == wk.default_host_settings().FilePath  # no trailing '/'
    assert host.CriticWeightFileName == b"critic" and host.ActorWeightFileName == b"actor"
    assert cfg.CriticNeuralNetwork == CRITIC.encode() and cfg.ActorNeuralNetwork == ACTOR.encode()
    assert fixes == [
        "Invalid file path for the program. (file path is invalid)",
        "Invalid file names. (actor weights file name is invalid; critic weights file name is invalid)",
        "Invalid neural networks. actor last dense layer should output 4, currently outputs 2; "
        "critic neural network not valid, check syntax",
    ]


def test_valid_nondefault_network_kept_then_rejected_by_create(wk):
    """The reference accepts any valid DSL; the kernels implement only the defaults, so
    wk_create refuses it (before touching a device) instead of running another net."""
    other = "Input |32| (ReLU) |32| (TanH) |1| Output"
    cfg, host, fixes = wk.config_from_json('{"CriticNeuralNetwork": "%s"}' % other)
    assert fixes == [] and cfg.CriticNeuralNetwork == other.encode()
    lib = wk.load_library()
    h = C.c_void_p()
    rc = lib.wk_create(C.byref(cfg), 0, 4, 1, C.byref(h))
    assert rc == -3 and b"unsupported" in lib.wk_last_error(None)


def test_string_escaping_round_trip(wk, tmp_path):
    d = tmp_path / "dir <&'+`> é 😀"
    d.mkdir()
    host = wk.default_host_settings()
    host.FilePath = (str(d) + "/").encode()
    host.CriticWeightFileName = 'q"uote\\back\ttab'.encode()
    text = wk.config_to_json(None, host)
    # JavaScriptEncoder.Default: HTML-sensitive characters and all non-ASCII as \uXXXX
    assert r"dir \u003C\u0026\u0027\u002B\u0060\u003E \u00E9 \uD83D\uDE00/" in text
    assert r'"q\u0022uote\\back\ttab"' in text
    _, host2, fixes = wk.config_from_json(text)
    assert fixes == [] and host2.FilePath == host.FilePath
    assert host2.CriticWeightFileName == host.CriticWeightFileName


def test_files_and_bom(wk, tmp_path):
    cfg = wk.default_config(Epochs=12, Gamma=0.99, UseGAE=1)
    host = wk.default_host_settings()
    p = tmp_path / "cfg.json"
    lib = wk.load_library()
    assert lib.wk_config_save_json(str(p).encode(), C.byref(cfg), C.byref(host)) == 0
    assert p.read_text(encoding="utf-8") == wk.config_to_json(cfg, host)
    p.write_bytes(b"\xef\xbb\xbf" + p.read_bytes())  # UTF-8 BOM, as .NET editors write
    cfg2, host2 = wk.default_config(), wk.default_host_settings()
    assert lib.wk_config_load_json(str(p).encode(), C.byref(cfg2), C.byref(host2)) == 0
    assert (cfg2.Epochs, cfg2.Gamma, cfg2.UseGAE) == (12, np.float32(0.99), 1)
    assert lib.wk_config_load_json(str(tmp_path / "none.json").encode(), C.byref(cfg2),
                                   C.byref(host2)) == -1
