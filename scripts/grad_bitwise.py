"""Gradient-kernel A/B bit-equality probe: minibatch gradients at several sizes (1..4 chunks
per wave, ragged, one skipped sample) and the weights after one whole wk_ppo_update, saved to
an .npz (WK_LIB picks the library); `compare a.npz b.npz` reports the first difference.
A re-scheduled kernel (same MFMA chains per accumulator, same VALU ops) must match bit for bit."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))

def run(out):
    import wk
    F = np.float32
    res = {}
    eng = wk.Engine(4, seed=20250905)
    for B in (16, 37, 2048, 8192, 20011, 65536):
        rng = np.random.default_rng(B)
        S = rng.normal(0, 1, (B, 12)).astype(F); A = rng.normal(0, 1, (B, 4)).astype(F)
        L = rng.normal(-3, 1, (B, 4)).astype(F); G = rng.normal(0, 5, B).astype(F)
        Ad = rng.normal(0, 1, B).astype(F)
        if B > 100: L[B // 3, 1] = -200.0
        g, cd, ad, sk = eng.minibatch_gradient(S, A, L, G, Ad)
        res[f"g{B}"] = np.concatenate([g, np.array([cd, ad, sk], F)])
    eng.close()
    n, T = 8192, 64
    eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=8192, Epochs=2)
    eng.rollout(T)
    eng.ppo_update(update_index=0)
    res["w_update"] = eng.get_weights()
    np.savez(out, **res)
    print("saved", out)

def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        x, y = A[k], B[k]
        if not np.array_equal(x.view(np.uint32), y.view(np.uint32)):
            i = np.flatnonzero(x.view(np.uint32) != y.view(np.uint32))
            print(f"{k}: {i.size} differ, first {i[0]}: {x[i[0]]!r} vs {y[i[0]]!r}, max abs {np.abs(x - y).max():.3g}")
            ok = False
        else:
            print(f"{k}: bit-identical")
    sys.exit(0 if ok else 1)

if __name__ == "__main__":
    if sys.argv[1] == "compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
