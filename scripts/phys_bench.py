"""Physics-kernel microbenchmark: rollout (policy fused) vs physics-only env-steps.

  python scripts/phys_bench.py [n_walkers] [T] [lanes...]
Prints ms per launch and env-steps/s for each lane mapping.  WK_SCENE=1: with the four scene
props of tests/test_gpu_scene.py (scene_a; the one-lane scene kernel).  WK_ROUGH=1: RoughFloor.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import torch  # noqa: E402
import wk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
lanes = [int(x) for x in sys.argv[3:]] or [1, 2, 16]
for L in lanes:
    eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, LanesPerWalker=L,
                    RoughFloor=int(os.environ.get("WK_ROUGH", "0")))
    if os.environ.get("WK_SCENE"):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_gpu_scene import scene_a
        eng.set_scene(scene_a(wk.make_prop))
    g = torch.Generator(device="cuda").manual_seed(1)
    act = torch.rand((T, n, 4), device="cuda", generator=g) * 2 - 1
    rew = torch.empty((T, n), device="cuda")
    done = torch.empty((T, n), device="cuda", dtype=torch.uint8)
    eng.rollout(T)
    eng.step_device(act.data_ptr(), T, None, rew.data_ptr(), done.data_ptr(), None)
    eng.sync()
    res = {}
    for name, fn in (("rollout", lambda: eng.rollout(T)),
                     ("physics", lambda: eng.step_device(act.data_ptr(), T, None, rew.data_ptr(),
                                                         done.data_ptr(), None))):
        reps = 3
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        eng.sync()
        dt = (time.perf_counter() - t0) / reps
        res[name] = dt
    print(f"L={L:2d} n={n} T={T}: rollout {res['rollout']*1e3:8.2f} ms "
          f"({n*T/res['rollout']/1e6:6.2f} M env-steps/s)  physics-only {res['physics']*1e3:8.2f} ms "
          f"({n*T/res['physics']/1e6:6.2f} M)", flush=True)
    eng.close()
