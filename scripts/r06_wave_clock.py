"""Per-wave start / end of one rollout launch (probe build: scripts/variant.sh wclk
"-DWK_WAVE_CLOCK" wk_physics.hip): in the bench regime (REGIME_ITERS PPO iterations at T_h 64
from the seeded start), how long each wave of the pair kernel runs, how far the last wave ends
after the mean one, and the spread by XCD -- the launch's tail, i.e. what a perfectly balanced
assignment of walkers to waves could recover.
  WK_LIB=ppo-bipedalwalker_amd/libwk_wclk.so python scripts/r06_wave_clock.py [walkers]"""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_wclk.so"))
import wk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R = int(os.environ.get("REGIME_ITERS", "8"))
eng = wk.Engine(n, seed=20250905, Horizon=64, RandomizeStart=1, Minibatch=min(n, 65536),
                MinibatchGlobal=65536)
lib = eng.lib
lib.wk_wave_clock.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * (4 * 8192))()
def lane_order(ep0):
    """wk_order.hip restated: the m episode-0 walkers take the last m slots, the r-th episode-0
    walker of the head trading places with the r-th post-reset walker of the tail"""
    n_ = ep0.size
    m = int(ep0.sum())
    order = np.arange(n_)
    h = np.flatnonzero(ep0[: n_ - m])
    t = (n_ - m) + np.flatnonzero(~ep0[n_ - m:])
    order[h], order[t] = t, h
    return order


for it in range(R + 3):
    st0 = eng.get_state() if it >= R else None
    eng.rollout(64)
    eng.sync()
    lib.wk_wave_clock(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4).astype(np.int64)
    waves = eng.rollout_mapping()["waves_launched"]
    a = a[:waves]
    t0, t1 = a[:, 0], a[:, 1]
    dur = (t1 - t0) / 100.0  # us (100 MHz)
    span = (t1.max() - t0.min()) / 100.0
    ends = (t1 - t0.min()) / 100.0
    xcc = a[:, 3] & 0xF
    line = (f"it {it}: waves {waves} span {span / 1e3:.2f} ms | wave duration mean {dur.mean() / 1e3:.2f} "
            f"p50 {np.median(dur) / 1e3:.2f} p90 {np.percentile(dur, 90) / 1e3:.2f} p99 "
            f"{np.percentile(dur, 99) / 1e3:.2f} max {dur.max() / 1e3:.2f} ms | start spread "
            f"{(t0.max() - t0.min()) / 100.0:.1f} us | mean/span {dur.mean() / span:.3f}")
    print(line, flush=True)
    if it >= R:
        per = ", ".join(f"x{x}: {dur[xcc == x].mean() / 1e3:.2f}/{dur[xcc == x].max() / 1e3:.2f}"
                        for x in range(8) if (xcc == x).any())
        print(f"   per XCD mean/max ms: {per}", flush=True)
        # waves by their slot in the lane order (wave index = slots 32 w .. 32 w + 31)
        q = np.array_split(dur, 8)
        print("   by wave-index octile (lane order), mean ms: " +
              " ".join(f"{x.mean() / 1e3:.2f}" for x in q), flush=True)
        tag = {"0": "unpaced", "2": "paced_nolayer"}.get(os.environ.get("WK_PACE", ""), "paced") + \
            ("_identity" if os.environ.get("WK_ORDER") == "0" else "")
        np.save(os.path.join(ROOT, "gpurun_out", f"wave_clock_{n}_{tag}_it{it}.npy"), a)
        if eng.rollout_mapping()["lanes_per_walker"] == 2 and os.environ.get("WK_ORDER") != "0":
            ep0 = st0[:, 109] == 0.0
            order = lane_order(ep0)
            wpw = 32
            steps = st0[order, 108].reshape(-1, wpw)
            e0 = ep0[order].reshape(-1, wpw)
            slow = np.argsort(dur)[-40:]
            fast = np.argsort(dur)[:1000]
            print(f"   episode-0 walkers {int(ep0.sum())}; slow waves: ep0/wave {e0[slow].mean(1).mean():.2f}, "
                  f"episode steps {steps[slow].mean():.0f}; other waves holding ep0: "
                  f"{[(int(w), round(float(dur[w]) / 1e3, 2), round(float(steps[w].mean()))) for w in np.flatnonzero(e0.any(1))[:60:4]]}",
                  flush=True)
            np.save(os.path.join(ROOT, "gpurun_out", f"wave_state_{n}_{tag}_it{it}.npy"), st0[order, 100:112])
    if it < R:
        eng.ppo_update(update_index=it, sync=False)
