"""PPO-update timing A/B: for each (walkers, minibatch, minibatch_global) shape a context runs
two PPO iterations, snapshots, rolls out once more, then times `reps` updates of that
trajectory (restore -> update; one HIP-event pair per update).  The library is whatever WK_LIB
names (run once per build).  Prints ms per update and us per minibatch.

  WK_LIB=.../libwk.so python scripts/update_ab.py [reps]
  UPDATE_SHAPES="32768:32768:65536,16384:16384:65536" selects other (walkers:M:M_global) shapes
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
T, E = 64, 5
SHAPES = ((65536, 65536, 65536), (8192, 8192, 65536), (4096, 4096, 4096))
if os.environ.get("UPDATE_SHAPES"):
    SHAPES = tuple(tuple(int(v) for v in sh.split(":")) for sh in os.environ["UPDATE_SHAPES"].split(","))
for n, M, Mg in SHAPES:
    eng = wk.Engine(n, seed=20250905, Horizon=T, Minibatch=M, MinibatchGlobal=Mg, Epochs=E,
                    RandomizeStart=1)
    for it in range(2):
        eng.rollout(T)
        eng.ppo_update(update_index=it, sync=False)
    eng.snapshot()
    eng.rollout(T)
    eng.ppo_update(update_index=2, sync=False)  # warm
    eng.profile_reset()
    eng.profile_enable(1)
    for _ in range(reps):
        eng.restore()
        eng.ppo_update(update_index=2, sync=False)
    p = eng.profile()
    eng.profile_enable(0)
    ms = p["update_ms"] / max(1, p["update_calls"])
    nmb = E * (n * T // M)
    print(f"{os.path.basename(os.environ.get('WK_LIB', 'libwk.so'))} n={n} M={M}: update {ms:.3f} ms "
          f"({ms * 1e3 / nmb:.2f} us per minibatch, {eng.grad_kernel(M)})", flush=True)
    eng.close()
