"""VERDICT r5 #2, counted: can the 8,192-walker shard's replay lanes speculate a leg's next pair?

The quad mapping at the 8-GPU shard holds 8 walkers per wave (one wave per SIMD; the other 32
lanes replay them).  A leg's chain per substep (Environment.cs:126-143, RigidBody.cs:54-96) is
integrate(lower) -> [floor] -> pair(lower, upper) -> [floor] -> integrate(upper) -> [floor] ->
pair(upper, lower) -> [floor].  Speculation would run integrate(upper) + SAT(upper, lower) on the
replay lanes while the owner lanes resolve the lower segment's pairs, and commit when those pairs
moved nothing: no leg-leg collision from the lower segment and no collision of the lower segment
with the floor (a box hit alone only sets Collided).  A wave can skip the sequential path only
when EVERY leg chain of its walkers commits -- otherwise it runs the redo (masked) after the
speculative pass, i.e. strictly more issue than today.  This counts, in the bench regime (8 PPO
iterations at T_h 64 from the seeded start, then policy env-steps traced per substep), the share
of walker-substeps and of wave-substeps (8 consecutive walkers = one wave of the sparse quad
mapping) in which the speculation would commit.

usage (GPU box): python3 scripts/r06_spec_commit.py [walkers] [env-steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import numpy as np  # noqa: E402
import wk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
eng = wk.Engine(n, seed=20250905, Horizon=64, Minibatch=n, MinibatchGlobal=65536, RandomizeStart=1)
for it in range(8):
    eng.rollout(64)
    eng.ppo_update(update_index=it)
mp = eng.rollout_mapping()
wpw = mp["walkers_per_wave"]
walker_ok, wave_ok, ll_rate, lf_rate = [], [], [], []
for k in range(K):
    _, act, _ = eng.policy_sample(eng.get_obs())
    tr = eng.step_traced(act)               # [n, Iterations]
    sat = tr["sat_hit"].astype(bool)        # [n, 50, 9]
    # pair slots (csrc/wk_physics.hip substep_side): left leg 0 lower-upper, 1 lower-floor,
    # right leg 5 lower-upper, 6 lower-floor
    inval = sat[:, :, [0, 1]].any(-1) | sat[:, :, [5, 6]].any(-1)   # either leg's lower pairs moved it
    ok = ~inval                                                     # [n, 50]
    walker_ok.append(ok.mean())
    ll_rate.append(sat[:, :, [0, 5]].mean())
    lf_rate.append(sat[:, :, [1, 6]].mean())
    waves = ok[: n // wpw * wpw].reshape(n // wpw, wpw, -1).all(axis=1)  # every walker of the wave
    wave_ok.append(waves.mean())
out = {"walkers": n, "walkers_per_wave": wpw, "env_steps_traced": K,
       "leg_leg_collision_rate_lower_slot": float(np.mean(ll_rate)),
       "lower_leg_floor_collision_rate": float(np.mean(lf_rate)),
       "walker_substep_commit_share": float(np.mean(walker_ok)),
       "wave_substep_commit_share": float(np.mean(wave_ok)),
       "note": ("commit = no leg-leg collision from either lower segment and no lower-segment floor "
                "collision in that substep; a wave skips the sequential pass only if all its walkers "
                "commit")}
print(json.dumps(out, indent=1))
