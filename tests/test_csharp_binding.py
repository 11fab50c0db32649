"""CPU: the C# P/Invoke binding (ppo-bipedalwalker_amd/cs/NativeMethods.cs) against the C ABI.

No .NET SDK exists in this container or on the GPU box, so the C# host
cannot be compiled here.  What can be checked is the part that breaks silently at run time:
every entry point of include/wk_api.h is declared, with the header's parameter count and,
per parameter, a marshalling of the right kind (pointer / array / ref / out vs. value, and
the value's width); every struct's sequential layout (size and field offsets) equals the
ctypes layout that tests/test_boundary.py checks against the library.
"""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "ppo-bipedalwalker_amd", "cs", "NativeMethods.cs")
HDR = os.path.join(ROOT, "include", "wk_api.h")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def header_prototypes():
    s = _strip_c_comments(open(HDR).read())
    out = {}
    for m in re.finditer(r"^\s*(?:int|void|const char\*)\s+(wk_\w+)\s*\(([^;]*?)\)\s*;", s, re.M):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",")]
        params = [] if params == ["void"] else params
        out[m.group(1)] = params
    return out


def cs_imports():
    s = open(CS).read()
    out = {}
    for m in re.finditer(r"\[DllImport\([^\]]*\)\]\s*public static extern\s+([\w\[\]?]+)\s+(wk_\w+)\s*\(([^;]*?)\);", s, re.S):
        params = [p.strip() for p in m.group(3).replace("\n", " ").split(",") if p.strip()]
        out[m.group(2)] = (m.group(1), params)
    return out


def c_kind(p):
    """the marshalling class of one C parameter"""
    if "*" in p or p.startswith("wk_host_allreduce_fn"):
        return "ptr"
    t = p.split()[0:-1]
    t = " ".join(t)
    return {"int": "i32", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
            "float": "f32", "double": "f64", "size_t": "usize"}[t]


def cs_kind(p):
    p = re.sub(r"\[(Out|In)\]\s*", "", p)
    toks = p.split()
    if toks[0] in ("ref", "out"):
        return "ptr"
    t = toks[0]
    if t.endswith("[]") or t.endswith("[]?") or t in ("IntPtr", "string", "HostAllReduce"):
        return "ptr"
    return {"int": "i32", "uint": "u32", "ulong": "u64", "long": "i64", "float": "f32", "double": "f64",
            "UIntPtr": "usize"}[t]


def test_every_export_is_declared_with_matching_signature():
    hdr = header_prototypes()
    cs = cs_imports()
    import wk
    assert set(hdr) == set(wk.EXPORTS), set(hdr) ^ set(wk.EXPORTS)
    missing = set(hdr) - set(cs)
    assert not missing, f"not declared in NativeMethods.cs: {sorted(missing)}"
    assert not set(cs) - set(hdr)
    for name, params in hdr.items():
        ret, cparams = cs[name]
        assert len(cparams) == len(params), (name, params, cparams)
        for cp, hp in zip(cparams, params):
            assert cs_kind(cp) == c_kind(hp), (name, hp, cp)
        assert ret in ("int", "void", "IntPtr"), (name, ret)


# C# sequential layout of the structs in NativeMethods.cs
_SIZES = {"int": 4, "uint": 4, "float": 4, "double": 8, "long": 8, "ulong": 8, "IntPtr": 8,
          "byte": 1}


def cs_struct_layouts():
    s = open(CS).read()
    out = {}
    for m in re.finditer(r"public (?:unsafe )?struct (\w+)\s*\{(.*?)\n\}", s, re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = re.sub(r"//.*", "", line).strip()
            if not line.startswith(("public", "[")):
                continue
            size_const = re.search(r"SizeConst\s*=\s*(\d+)", line)
            line = re.sub(r"^\[[A-Za-z][^\]]*\]\s*", "", line)
            toks = line.replace(",", " , ").split()
            assert toks[0] == "public"
            if toks[1] == "fixed":
                t = toks[2]
                name, n = re.match(r"(\w+)\[(\d+)\]", toks[3]).groups()
                fields.append((name, _SIZES[t], _SIZES[t] * int(n)))
                continue
            t = toks[1]
            names = [x for x in toks[2:] if x != ","]
            for nm in names:
                if t == "string":
                    fields.append((nm, 1, int(size_const.group(1))))
                else:
                    fields.append((nm, _SIZES[t], _SIZES[t]))
        off, al, lay = 0, 1, []
        for nm, a, sz in fields:
            off = (off + a - 1) // a * a
            lay.append((nm, off, sz))
            off += sz
            al = max(al, a)
        out[m.group(1)] = (lay, (off + al - 1) // al * al)
    return out


@pytest.mark.parametrize("cs_name,py_name", [
    ("WkConfig", "WkConfig"), ("WkHostSettings", "HostSettings"), ("WkPairTrace", "PairTrace"),
    ("WkBodyView", "BodyView"), ("WkProp", "Prop"), ("WkPropView", "PropView"),
    ("WkPpoArgs", "PpoArgs"), ("WkRolloutStats", "RolloutStats"), ("WkEpisodeRec", "EpisodeRec"),
    ("WkProfile", "Profile")])
def test_struct_layouts_match_ctypes(cs_name, py_name):
    import wk
    lay, size = cs_struct_layouts()[cs_name]
    py = getattr(wk, py_name)
    assert size == C.sizeof(py), (cs_name, size, C.sizeof(py))
    py_offsets = [(f[0], getattr(py, f[0]).offset, getattr(py, f[0]).size) for f in py._fields_]
    assert [(o, s) for _, o, s in lay] == [(o, s) for _, o, s in py_offsets], (lay, py_offsets)


def test_headless_environment_uses_the_sampled_step():
    """the C# Environment.Update fills the Trajectory from wk_step_sampled (unclipped actions
    and log-probabilities, Environment.cs:74-89) and trains through wk_set_trajectory +
    wk_ppo_update (PPOAgent.Train(Trajectory))"""
    src = open(os.path.join(ROOT, "ppo-bipedalwalker_amd", "cs", "HeadlessEnvironment.cs")).read()
    for call in ("wk_step_sampled", "wk_set_trajectory", "wk_ppo_update", "wk_get_body_view"):
        assert f"Wk.{call}(" in src
