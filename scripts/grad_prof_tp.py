"""Phase profile of k_ppo_grad_tp (build: bash scripts/variant.sh gprof -DWK_GRAD_PROF
wk_ppo_mfma.hip): s_memtime cycles of wave 0 of each block (team 0, tile 0), averaged over
blocks and launches, per minibatch size.  WK_GRAD_IMPL = tp / tp1.
  python scripts/grad_prof_tp.py [sizes]"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_gprof.so"))
import wk  # noqa: E402

names = ["prologue", "layer1", "B1 wait", "layer2+rows", "B2 wait", "loss+VALU", "B3 wait",
         "backward", "row sums", "slab"]
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,8192,65536").split(",")]
teams = 1 if os.environ.get("WK_GRAD_IMPL") == "tp1" else 2
n, T = 65536, 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=1)
lib = eng.lib
lib.wk_grad_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 16)()
eng.rollout(T)
eng.ppo_update(minibatch=n, update_index=0)
eng.sync()
for M in sizes:
    lib.wk_grad_prof(buf, 1)
    eng.ppo_update(minibatch=M, update_index=1)
    eng.sync()
    lib.wk_grad_prof(buf, 1)
    launches = (n * T) // M
    chunks = (M + 15) // 16
    blocks = min(256, (chunks + teams - 1) // teams)
    cpt = chunks / (blocks * teams)
    tot = sum(buf[i] for i in range(10)) / (blocks * launches)
    print(f"M={M} teams={teams}: {launches} launches x {blocks} blocks, {cpt:.2f} chunks/team, "
          f"wave-0 lifetime {tot:.0f} cycles", flush=True)
    for i, nm in enumerate(names):
        v = buf[i] / (blocks * launches)
        per = f"  {v / cpt:8.0f} per chunk" if 1 <= i <= 7 else ""
        print(f"  {nm:12s} {v:9.0f} cycles{per}")
