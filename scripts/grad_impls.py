"""A/B of the matrix-core gradient kernels (WK_GRAD_IMPL = ws / tp / tp1 / mf): the gradient
kernel's mean launch time (burst of 64 on minibatch 0, wk_time_gradient) and one whole PPO
update (E = 5, 320 minibatches) per minibatch size.  Also checks that every kernel gives the
same weights within fp32 association noise.

  python scripts/grad_impls.py [impls] [walkers,...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk  # noqa: E402

impls = (sys.argv[1] if len(sys.argv) > 1 else "ws,tp,tp1").split(",")
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4096,8192,16384,65536").split(",")]
T = 64
for n in sizes:
    ref_w = None
    for impl in impls:
        os.environ["WK_GRAD_IMPL"] = impl
        eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=5)
        eng.rollout(T)
        eng.sync()
        g_ms = eng.time_gradient(0, 64)
        w0, adam0 = eng.get_weights(), eng.get_adam()
        eng.ppo_update(update_index=0)  # warm
        eng.set_weights(w0)
        eng.set_adam(*adam0)
        eng.sync()
        t0 = time.perf_counter()
        eng.ppo_update(update_index=0)
        eng.sync()
        u_ms = (time.perf_counter() - t0) * 1e3
        w = eng.get_weights()
        d = "" if ref_w is None else f"  max|dw| vs {impls[0]} {np.abs(w - ref_w).max():.3g}"
        if ref_w is None:
            ref_w = w
        print(f"walkers {n:6d} impl {impl:4s} grad {g_ms * 1e3:7.2f} us  update {u_ms:7.3f} ms{d}",
              flush=True)
        eng.close()
