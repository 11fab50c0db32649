"""Weights-file format, through the C ABI with no GPU.

The reference writes one text file per network (PPOAgent.Save PPOAgent.cs:192-213):
line 0 the network DSL string (NeuralNetwork.Save NeuralNetwork.cs:159-176), then one
line per dense layer "W <weights row-major> B <biases>" (DenseLayer.Save DenseLayer.cs:73-79,
Matrix.Save Matrix.cs:133-153, values joined by single spaces with float.ToString()).

The reference ships no .weights files, so the digit strings are pinned by .NET Core 3.0+'s
documented float formatting (shortest round-trip digits, General format switching to
"E+XX" when the decimal-point position exceeds max(digits, 9) or is below -3) and checked
against numpy's independent shortest-digit algorithm -- "parity unpinned" against a real
.NET run, which this image cannot make.
"""
import numpy as np
import pytest

CRITIC_DSL = "Input |64| (LeakyReLU) |1| Output"
ACTOR_DSL = "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output"
# (rows, cols) of each dense layer, reference DenseLayer order
CRITIC_LAYERS = [(64, 12), (1, 64)]
ACTOR_LAYERS = [(64, 12), (64, 64), (4, 64)]


@pytest.mark.parametrize("value,text", [
    (0.0, "0"), (-0.0, "-0"), (1.0, "1"), (-60.0, "-60"), (1.5, "1.5"), (0.1, "0.1"),
    (0.3, "0.3"), (1 / 3, "0.33333334"), (1e-3, "0.001"), (1e-4, "0.0001"), (1e-5, "1E-05"),
    (1.2345e-5, "1.2345E-05"), (16777216.0, "16777216"), (1e8, "100000000"),
    (123456789.0, "123456790"), (1e9, "1E+09"), (3.4028235e38, "3.4028235E+38"),
    (1e-45, "1E-45"), (float("inf"), "∞"), (float("-inf"), "-∞"), (float("nan"), "NaN"),
])
def test_dotnet_float_strings(wk, value, text):
    p = np.zeros(wk.NPARAM, np.float32)
    p[0] = value
    critic, _ = wk.format_weights(p)
    assert critic.split("\n")[1].split(" ")[1] == text


def _layout(wk, p):
    """the WK_NPARAM vector cut into the reference's per-layer (W, B) matrices"""
    off = 0
    out = []
    for layers in (CRITIC_LAYERS, ACTOR_LAYERS):
        net = []
        for r, c in layers:
            w = p[off:off + r * c].reshape(r, c)
            off += r * c
            b = p[off:off + r]
            off += r
            net.append((w, b))
        out.append(net)
    assert off == wk.NPARAM
    return out


def test_file_structure_matches_reference(wk):
    rng = np.random.default_rng(1)
    p = rng.standard_normal(wk.NPARAM).astype(np.float32)
    critic, actor = wk.format_weights(p)
    for text, dsl, net in zip((critic, actor), (CRITIC_DSL, ACTOR_DSL), _layout(wk, p)):
        lines = text.split("\n")
        assert lines[-1] == ""  # File.WriteAllLines terminates every line
        lines = lines[:-1]
        assert lines[0] == dsl and len(lines) == len(net) + 1
        for line, (w, b) in zip(lines[1:], net):
            head, tail = line.split(" B ")
            assert head.startswith("W ")
            ws = np.array(head[2:].split(" "), dtype=np.float32)
            bs = np.array(tail.split(" "), dtype=np.float32)
            np.testing.assert_array_equal(ws, w.ravel())  # row-major, Matrix.cs:139-153
            np.testing.assert_array_equal(bs, b)


def test_shortest_digits_agree_with_numpy(wk):
    """every token has exactly the significant digits of numpy's shortest round-trip repr"""
    rng = np.random.default_rng(2)
    bits = rng.integers(0, 2**32, wk.NPARAM, dtype=np.uint64).astype(np.uint32)
    p = bits.view(np.float32).copy()
    p[~np.isfinite(p)] = 1.0
    critic, actor = wk.format_weights(p)
    toks = []
    for text in (critic, actor):
        for line in text.split("\n")[1:-1]:
            toks += [t for t in line.split(" ") if t not in ("W", "B")]
    assert len(toks) == wk.NPARAM
    order = np.concatenate([np.concatenate([np.r_[w.ravel(), b] for w, b in net])
                            for net in _layout(wk, np.arange(wk.NPARAM, dtype=np.float64))])
    for tok, idx in zip(toks, order.astype(np.int64)):
        v = p[idx]
        sci = np.format_float_scientific(v, unique=True, trim="-")
        mant = sci.split("e")[0].lstrip("-").replace(".", "")
        digits = tok.lstrip("-").split("E")[0].replace(".", "").lstrip("0").rstrip("0") or "0"
        assert digits == mant.rstrip("0") or (mant.rstrip("0") == "" and digits == "0"), (tok, sci)
        assert np.float32(tok) == v


def _tokens(wk, p):
    critic, actor = wk.format_weights(p)
    toks = []
    for text in (critic, actor):
        for line in text.split("\n")[1:-1]:
            toks += [t for t in line.split(" ") if t not in ("W", "B")]
    order = np.concatenate([np.concatenate([np.r_[w.ravel(), b] for w, b in net])
                            for net in _layout(wk, np.arange(wk.NPARAM, dtype=np.float64))])
    out = [None] * wk.NPARAM
    for tok, idx in zip(toks, order.astype(np.int64)):
        out[idx] = tok
    return out


def test_shortest_digits_at_binade_edges(wk):
    """Powers of two (asymmetric round-trip interval) and their neighbours, normal and
    subnormal: the digits equal numpy's shortest unique repr (Dragon4)."""
    ex = np.arange(1, 255, dtype=np.uint32) << 23
    sub = np.uint32(1) << np.arange(23, dtype=np.uint32)
    base = np.concatenate([ex, sub])
    bits = np.concatenate([base, base + 1, base - 1, base | 0x80000000])
    bits = bits[(bits & 0x7F800000) != 0x7F800000]
    p = np.ones(wk.NPARAM, np.float32)
    p[:bits.size] = bits.view(np.float32)
    toks = _tokens(wk, p)
    for i in range(bits.size):
        v = p[i]
        sci = np.format_float_scientific(v, unique=True, trim="-")
        mant, e = sci.split("e")
        tok = toks[i]
        assert np.float32(tok) == v, (tok, sci)
        digits = tok.lstrip("-").split("E")[0].replace(".", "").lstrip("0").rstrip("0")
        assert digits == mant.lstrip("-").replace(".", "").rstrip("0"), (tok, sci)


def test_round_trip_bitexact(wk):
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 2**32, wk.NPARAM, dtype=np.uint64).astype(np.uint32)
    p = bits.view(np.float32).copy()
    p[np.isnan(p)] = -0.0
    p[:4] = [np.inf, -np.inf, 1e-45, -3.4028235e38]
    q = wk.parse_weights(*wk.format_weights(p))
    np.testing.assert_array_equal(p.view(np.uint32), q.view(np.uint32))


def test_parse_accepts_crlf_and_dotnet_spellings(wk):
    p = np.random.default_rng(4).standard_normal(wk.NPARAM).astype(np.float32)
    critic, actor = wk.format_weights(p)
    q = wk.parse_weights(critic.replace("\n", "\r\n"), actor.replace("\n", "\r\n"))
    np.testing.assert_array_equal(p, q)
    lines = critic.split("\n")
    toks = lines[2].split(" ")
    toks[1] = "Infinity"  # invariant-culture spelling
    lines[2] = " ".join(toks)
    q = wk.parse_weights("\n".join(lines), actor)
    assert q[768 + 64] == np.inf


def _mutate(text, line, fn):
    lines = text.split("\n")
    lines[line] = fn(lines[line])
    return "\n".join(lines)


@pytest.mark.parametrize("case", ["dsl", "short", "token", "missing", "extra", "double_space",
                                  "no_bias"])
def test_parse_rejects_malformed(wk, case):
    """NeuralNetwork.Load / ValidateWeights (NeuralNetwork.cs:94-157) refuse these; the
    reference then silently keeps its weights, the C ABI returns an error instead."""
    p = np.random.default_rng(5).standard_normal(wk.NPARAM).astype(np.float32)
    critic, actor = wk.format_weights(p)
    bad = {
        "dsl": lambda: _mutate(critic, 0, lambda s: s.replace("64", "32")),
        "short": lambda: "\n".join(critic.split("\n")[:2]),
        "token": lambda: _mutate(critic, 1, lambda s: s.replace(" ", " x", 1)),
        "missing": lambda: _mutate(critic, 1, lambda s: s.split(" B ")[0].rsplit(" ", 1)[0]
                                   + " B " + s.split(" B ")[1]),
        "extra": lambda: _mutate(critic, 2, lambda s: s + " 1"),
        "double_space": lambda: _mutate(critic, 1, lambda s: s.replace(" ", "  ", 3)),
        "no_bias": lambda: _mutate(critic, 2, lambda s: s.split(" B ")[0]),
    }[case]()
    with pytest.raises(wk.WkError):
        wk.parse_weights(bad, actor)
    q = wk.parse_weights(critic, actor)  # the intact pair still parses
    np.testing.assert_array_equal(p, q)
