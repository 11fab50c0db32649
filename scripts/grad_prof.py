"""Phase profile of k_ppo_grad_mfma (build: bash scripts/variant.sh gprof -DWK_GRAD_PROF
wk_ppo_mfma.hip): s_memtime cycles of wave 0 per block, averaged over blocks and launches,
for one update pass at each minibatch size.  python scripts/grad_prof.py"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_gprof.so"))
import wk  # noqa: E402

names = ["prologue", "gather+SX", "layer1", "layer2", "out rows", "loss", "gz2+G2", "dW3/dW2",
         "gh1+gz1", "dW1", "loop exit", "epilogue"]
n, T = 65536, 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=1)
lib = eng.lib
lib.wk_grad_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 16)()
eng.rollout(T)
eng.ppo_update(minibatch=n, update_index=0)
eng.sync()
for M in (8192, 65536):
    lib.wk_grad_prof(buf, 1)
    eng.ppo_update(minibatch=M, update_index=1)
    eng.sync()
    lib.wk_grad_prof(buf, 1)
    launches = (n * T) // M
    chunks = (M + 15) // 16
    blocks = min(256, (chunks + 3) // 4)
    cpw = chunks / (blocks * 4)
    tot = sum(buf[i] for i in range(12)) / (blocks * launches)
    print(f"M={M}: {launches} launches x {blocks} blocks, {cpw:.2f} chunks/wave, "
          f"wave-0 lifetime {tot:.0f} cycles")
    for i, nm in enumerate(names):
        v = buf[i] / (blocks * launches)
        per = f"  {v / cpw:8.0f} per chunk" if 1 <= i <= 9 else ""
        print(f"  {nm:10s} {v:9.0f} cycles{per}")
