#!/usr/bin/env python3
"""bench.py -- batched bipedal-walker physics + PPO on MI355X (BASELINE.json metric).

One "step" = one PPO iteration over this rank's walkers: a device-resident rollout of
`--horizon` env-steps (policy sampling + 50 physics substeps + reward/terminal/auto-reset
+ value estimate, fused in one HIP kernel) followed by the returns scan and the PPO
update (E epochs x pool/M minibatches: gradient kernel -> ordered reduction -> RCCL
all-reduce -> Adam).

Workload (BASELINE.json configs[3]): 65,536 walkers in total, sharded over the N GPUs
(8,192 per GPU at N = 8), global minibatch 65,536 (M = 65,536 / N per GPU), T_h = 64, E = 5
-- `scaling: strong`.  At N = 1 that is the metric's 65,536 walkers on one MI355X.
`--walkers W` instead fixes W walkers per GPU (`scaling: weak`).

Regime: throughput depends on where training is (episode lengths change the reset / contact
mix), so the bench runs a fixed `--regime-iters` iterations from the seeded initial state,
snapshots the whole training state on the device (wk_snapshot), and every warm-up and timed
iteration restores it first (a ~30 MB device copy, inside the timed region): each timed
step is the same iteration, whatever --steps / --warmup the driver passes.

value = env-steps of all ranks / max-over-ranks wall time of the K timed steps.

  python bench.py [--gpus N --steps K --warmup W --walkers-global 65536 --horizon 64]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))

METRIC = "env-steps/sec (whole node) + PPO-update ms, 65k walkers at 1/2/4/8 MI355X"
# MI355X_MICROARCH.md: fp32 peak 157.3 TF (vector = matrix: v_mfma_f32_16x16x4_f32 runs at the
# vector rate), i.e. 1,024 SIMDs x 2.4 GHz x 64 flop/clk -- a wave64 v_fma_f32 (128 flop) every
# 2 cycles.  The physics is restated op for op with no FMA contraction (parity), so one VALU
# instruction is one flop per lane: its ceiling is the scalar non-FMA rate, 78.6 T op/s
# (a wave64 instruction per 2 cycles per SIMD), reachable once each SIMD holds >= 2 waves.
# With one wave per SIMD a wave issues one VALU instruction per 4 cycles (the guide's
# 'vector-instruction ISSUE cost' row): 39.3 T, scaled by the share of SIMDs that hold a wave.
PEAK_FP32_TFLOPS = 157.3
PEAK_NOFMA = 78.6
PEAK_NOFMA_ONE_WAVE = 39.3
N_SIMDS = 1024
PEAK_HBM_GBS = 8000.0
# SURVEY 8(d) PPO-update flop model: per sample and epoch, forward + backward of actor and
# critic (PPOAgent.cs:218-346, DenseLayer.cs:103-120); Adam ~14 flop x 6,149 per minibatch
FLOP_GRAD_SAMPLE = 36569
FLOP_ADAM_MINIBATCH = 86086
GRAD_BURST = 64  # back-to-back gradient launches timed for the update roofline
SLAB_BYTES = 6152 * 4  # gradient + 3 diagnostics, padded to 16 B: the all-reduce payload
# SURVEY.md 8(d) flop model, priced per counted physics event (wk_count_events):
FLOP_INTEGRATE = 477          # per walker-substep: 4 poles x 95 + hull 81 + floor 16
FLOP_JOINT = 107              # per Joint.Step past the 0.1 early-out ((2x106 + 2x108) / 4)
FLOP_SAT = {"ll": 571, "lf": 417, "bf": 349}       # (VA+VB)(11+3(VA+VB))+7, per AABB hit
FLOP_CONTACT = {"ll": 190, "lf": 166, "bf": 161}   # contact clipping + MoveObjects, per SAT hit
FLOP_IMPULSE = 110            # normal + friction impulse pair, per resolution with contacts
FLOP_POLICY = 10504 + 1793 + 130  # actor + critic forward, sampling / log-prob, obs / reward
FLOP_UPPER = 3.0e5            # SURVEY's all-pairs-colliding upper bound per env-step (flat floor:
                              # the rough floor's 11 segments give the counted F more pairs than it)
# algorithmic HBM bytes per env-step of the rollout: trajectory row 89 B +
# the 448-B walker record read and written once per T_h = 64 env-steps
def alg_bytes_per_env_step(horizon):
    return 89.0 + 2 * 448.0 / horizon


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--walkers-global", type=int, default=65536,
                   help="walkers over all GPUs (strong scaling, BASELINE config 4)")
    p.add_argument("--walkers", type=int, default=0,
                   help="walkers per GPU instead (weak scaling)")
    p.add_argument("--horizon", type=int, default=64)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--minibatch-global", type=int, default=0,
                   help="global minibatch (0 = all walkers: 65,536)")
    p.add_argument("--materials", action="store_true", help="config 5: random Ice/Rubber/Carpet")
    p.add_argument("--seed", type=int, default=20250905)
    p.add_argument("--lanes", type=int, default=0,
                   help="lanes per walker in the physics kernel (0 auto, 1, 2 or 16)")
    p.add_argument("--regime-iters", type=int, default=8,
                   help="PPO iterations from the seeded start before the snapshot")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the configs 2 / 3 / 4-shard / 5-shard lines (N = 1 only)")
    p.add_argument("--cpu-baseline-steps", type=int, default=150000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="processes of the all-cores CPU baseline (0: every CPU the process may use)")
    p.add_argument("--rehearse", action="store_true",
                   help="multi-rank rehearsal on ONE GPU: every rank on device 0, the exchange "
                        "either IPC (--exchange ipc, the default) or the host all-reduce over "
                        "gloo (wk_comm_init_host; RCCL refuses two ranks on one device) -- "
                        "exercises the N > 1 code path; not a performance number")
    p.add_argument("--exchange", choices=("rccl", "ipc"), default="ipc",
                   help="N > 1 minibatch gradient exchange: the one-shot exchange over IPC-mapped "
                        "peer memory fused with the ordered reduction and Adam (wk_comm_init_ipc; "
                        "checked bit for bit against a rank-order reference before timing, and "
                        "RCCL on every rank if the mapping, the test round or the check fails), "
                        "or the RCCL all-reduce")
    p.add_argument("--xch-profile", action="store_true",
                   help="N > 1 with the IPC exchange: after timing, one untimed iteration with the "
                        "exchange kernel's per-block clock stamps (wk_comm_xch_profile): wait for "
                        "peers versus own work per minibatch, in the detail file and the line")
    p.add_argument("--detail-file", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                   help="full result (every roofline field, event rates, notes); the stdout line "
                        "is the compact <= 4 KB summary and names this file ('' = do not write)")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_physics.json"))
    return p.parse_args()


# ---------------------------------------------------------------- CPU baseline ----------
_CPU_WORKER = """
import sys, time
sys.path.insert(0, sys.argv[1])
import orc
n, env, seed, t_start = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
orc.physics_loop(200, seed=seed, env=env)  # load + warm
while time.time() < t_start:
    time.sleep(0.001)
t0 = time.perf_counter()
orc.reference_loop(n, seed=seed, env=env)
print(time.perf_counter() - t0)
"""


def _all_cores(threads, n_each, seed):
    """one walker per process (the reference loop), all processes started together; child
    processes with no GPU (subprocess: fork + exec before anything touches a device)"""
    import subprocess
    t_start = time.time() + 2.0
    procs = [subprocess.Popen([sys.executable, "-c", _CPU_WORKER, os.path.join(ROOT, "oracle"),
                               str(n_each), str(i), str(seed), repr(t_start)],
                              stdout=subprocess.PIPE, text=True) for i in range(threads)]
    secs = [float(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
    if any(p.returncode for p in procs):
        raise RuntimeError("a CPU baseline worker failed")
    return threads * n_each / max(secs)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_quota():
    """CPUs the cgroup grants this process (cgroup v2 cpu.max, v1 cfs quota), or None"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(args):
    """the oracle (C restatement of the reference's single-threaded C#
    loop) on the host cores: (i) 1 walker on 1 core -- the full loop (policy + physics +
    Train at every episode end), physics only, and Train ms per 1001-step episode; (ii) one
    walker per process on the box's CPU share."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    orc.build()
    n = args.cpu_baseline_steps
    t0 = time.perf_counter()
    eps, train_s = orc.reference_loop(n, seed=args.seed)
    dt = time.perf_counter() - t0
    n_phys = max(1000, n // 2)
    t0 = time.perf_counter()
    orc.physics_loop(n_phys, seed=args.seed)
    dt_phys = time.perf_counter() - t0
    train_ms = min(orc.train_episode_seconds(1001, seed=args.seed) for _ in range(3)) * 1e3
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # one walker per process on every CPU this process may run on: the affinity set, capped by
    # the cgroup's CPU quota when it has one (more processes than granted CPUs only time-share)
    quota = _cpu_quota()
    threads = max(1, min(avail, int(quota)) if quota else avail)
    if args.cpu_threads:
        threads = args.cpu_threads
    why = (f"affinity {avail} CPUs" + (f", cgroup quota {quota:g} CPUs" if quota else ", no cgroup quota")
           + (" (overridden by --cpu-threads)" if args.cpu_threads else ""))
    n_each = max(1000, n // 4)
    all_rate = _all_cores(threads, n_each, args.seed)
    return {"value": n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": (f"{n} env-steps of the single-walker reference loop (policy + physics, "
                       f"PPO Train at each of {eps} episode ends: {train_s:.2f} s of {dt:.2f} s)"),
            "physics_only_env_steps_per_s": n_phys / dt_phys,
            "physics_only_sample": f"{n_phys} env-steps, one walker, uniform synthetic actions",
            "train_ms_per_1001_step_episode": train_ms,
            "all_cores": {"threads": threads, "env_steps_per_s": all_rate,
                          "sample": f"{threads} processes x {n_each} env-steps of the reference loop",
                          "nproc": os.cpu_count(), "affinity_cpus": avail, "cgroup_cpu_quota": quota,
                          "threads_reason": why, "cpu_model": _cpu_model()}}


# ---------------------------------------------------------------- GPU -------------------
GRAD_KERNEL_DESC = {"k_ppo_grad_ws": "producer/consumer waves",
                    "k_ppo_grad_tp": "tile-parallel teams of four waves, two per block",
                    "k_ppo_grad_tp1": "tile-parallel teams of four waves, one per block"}


def update_roofline(prof_k, samples_per_minibatch, walkers, horizon, epochs, update_ms, burst_ms,
                    burst_ev_ms, kernel, exchange="none"):
    """SURVEY 8(d) update roofline: the gradient kernel the update launches at this minibatch
    (wk_grad_kernel; one launch per minibatch) priced at 36,569 flop per sample over its mean
    duration INSIDE a real update: the per-launch HIP-event mean of one untimed
    update with an event pair around every launch (profile level 2), minus the per-launch event
    overhead measured on the same kernel (a burst of back-to-back launches timed with an event
    pair around every launch, minus the same burst timed by one pair) -- and the whole update
    (gradient + reduction + exchange + Adam over all minibatches) over its measured time"""
    launches = max(1, prof_k.get("grad_launches", 0))
    ev_mean_us = prof_k["grad_ms"] / launches * 1e3
    overhead_us = max(0.0, (burst_ev_ms - burst_ms) * 1e3)
    grad_us = ev_mean_us - overhead_us
    achieved = FLOP_GRAD_SAMPLE * samples_per_minibatch / (grad_us * 1e-6) / 1e12
    n_mb = epochs * (walkers * horizon // samples_per_minibatch)
    upd_flop = epochs * walkers * horizon * FLOP_GRAD_SAMPLE + n_mb * FLOP_ADAM_MINIBATCH
    upd_tf = upd_flop / (update_ms * 1e-3) / 1e12
    desc = GRAD_KERNEL_DESC.get(kernel, "")
    out = {"bound": "mfma", "kernel": f"{kernel} ({desc + ', ' if desc else ''}v_mfma_f32_16x16x4_f32)",
           "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
           "frac": achieved / PEAK_FP32_TFLOPS, "traffic": None,
           "samples_per_launch": samples_per_minibatch, "flop_per_sample": FLOP_GRAD_SAMPLE,
           "mean_launch_us": grad_us,
           "mean_launch_us_per_launch_events": ev_mean_us,
           "event_overhead_us": overhead_us,
           "burst_us": burst_ms * 1e3, "burst_launches": GRAD_BURST,
           "update": {"minibatches": n_mb, "flop": upd_flop, "ms": update_ms,
                      "achieved": upd_tf, "frac": upd_tf / PEAK_FP32_TFLOPS},
           "note": ("achieved = 36,569 flop/sample (SURVEY 8(d)) x samples per launch / the "
                    "gradient kernel's mean in-update duration: per-launch HIP events (engine "
                    "stream) over one real update's launches minus the per-launch event "
                    f"overhead ({overhead_us:.2f} us: {GRAD_BURST} back-to-back launches timed "
                    "per launch vs by one pair); burst_us is the warm back-to-back mean")}
    per = lambda k: prof_k[k + "_ms"] / max(1, prof_k.get(k + "_launches", prof_k.get(k + "_calls", 0))) * 1e3
    if exchange == "ipc":  # one fused launch per minibatch (profiled as the all-reduce)
        out["reduce_exchange_adam_us"] = prof_k["allreduce_ms"] / max(1, prof_k["allreduce_calls"]) * 1e3
    elif exchange in ("none",):
        out["reduce_adam_us"] = per("reduce")
    else:
        out["reduce_us"] = per("reduce")
        out["allreduce_us"] = prof_k["allreduce_ms"] / max(1, prof_k["allreduce_calls"]) * 1e3
        out["adam_us"] = per("adam")
    return out


def flops_per_env_step(ev, policy=True):
    """SURVEY 8(d)'s per-primitive constants priced on the counted events"""
    f = FLOP_INTEGRATE * ev["substeps"] + FLOP_JOINT * ev["joint"] + FLOP_IMPULSE * (
        ev["imp_ll"] + ev["imp_lf"] + ev["imp_bf"])
    for c in ("ll", "lf", "bf"):
        f += FLOP_SAT[c] * ev["aabb_" + c] + FLOP_CONTACT[c] * ev["sat_" + c]
    return f / ev["env_steps"] + (FLOP_POLICY if policy else 0)


def valu_ceiling_of(mapping):
    """the non-FMA VALU ceiling of a rollout launch from its real grid (wk_rollout_mapping):
    >= 2 waves per SIMD -> 78.6 T; else one wave per SIMD on the share of SIMDs holding one"""
    waves = mapping.get("waves_launched", mapping["waves"])  # idle waves of the last block run too
    if waves >= 2 * N_SIMDS:
        return PEAK_NOFMA, "scalar non-FMA fp32 issue, >= 2 waves per SIMD"
    return (PEAK_NOFMA_ONE_WAVE * min(1.0, waves / N_SIMDS),
            f"one wave per SIMD on {min(waves, N_SIMDS)} of {N_SIMDS} SIMDs "
            "(a wave64 VALU instruction per 4 cycles)")


KERNEL_OF_LANES = {2: "k_env_side<...,1> (pair mapping)", 4: "k_env_side<...,2> (quad mapping)",
                   16: "k_env_step<...,16> (16-lane rows)", 1: "k_env_step<...,1> (one lane per walker)"}


def rollout_roofline(eng, wk, launch_ms, units, horizon, policy=True, traffic=None):
    """the rollout kernel's roofline on THIS context: its physics events counted by replaying the
    timed iteration's actions (restore -> wk_count_events) and priced with SURVEY 8(d)'s
    constants, over the mean launch time (HIP events on the engine stream, profile level 1)"""
    eng.restore()
    ev = dict(zip(wk.EVENTS, eng.count_events(horizon).tolist()))
    f = flops_per_env_step(ev, policy)
    achieved = f * units / (launch_ms * 1e-3) / 1e12
    mp = eng.rollout_mapping()
    ceiling, why = valu_ceiling_of(mp)
    return {
        "bound": "valu",
        "kernel": (KERNEL_OF_LANES[mp["lanes_per_walker"]]
                   + (" fused rollout: physics + matrix-core policy" if policy else " physics only")),
        "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": achieved / PEAK_FP32_TFLOPS, "traffic": traffic,
        "peak_no_fma": ceiling, "frac_no_fma": achieved / ceiling, "peak_no_fma_basis": why,
        "mapping": mp,
        "flop_per_env_step_counted": f, "flop_per_env_step_upper_bound_flat_floor": FLOP_UPPER,
        "events_per_env_step": {k: v / ev["env_steps"] for k, v in ev.items() if k != "env_steps"},
        "env_steps_per_launch": units, "mean_launch_ms": launch_ms,
        "hbm_GBs": (traffic / (launch_ms * 1e-3) / 1e9) if traffic else None,
        "hbm_frac": (traffic / (launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS) if traffic else None,
        "alg_bytes_per_launch": (alg_bytes_per_env_step(horizon) if policy else 0.0) * units,
        "note": (f"VALU-issue bound (op-for-op fp32 restatement, no FMA contraction); achieved = "
                 f"F_counted {f:.0f} flop/env-step (SURVEY 8(d) constants priced on this "
                 f"iteration's counted AABB/SAT/contact/impulse/joint events) x {units:.0f} "
                 f"env-steps per launch / {launch_ms:.3f} ms mean launch (HIP events on the "
                 "engine stream)")}


def time_iterations(eng, args, k, horizon, update_index, barrier=None, physics_only=None):
    """k iterations, each restoring the snapshot; returns wall seconds"""
    if barrier:
        barrier()
    else:
        eng.sync()
    t0 = time.perf_counter()
    for _ in range(k):
        eng.restore()
        if physics_only is not None:
            physics_only()
        else:
            eng.rollout(horizon)
            eng.ppo_update(update_index=update_index, sync=False)
    if barrier:
        eng.sync()
        barrier()
    else:
        eng.sync()
    return time.perf_counter() - t0


def extra_config(wk, torch, args, n, M, M_global, horizon, physics_only=False, materials=False,
                 k=5, rough=False):
    """one of BASELINE's other shapes on this GPU (same regime protocol as the main line), with
    its own rollout roofline and update roofline; rough: the same loop on
    CreateRoughFloor's terrain"""
    eng = wk.Engine(n, seed=args.seed, Horizon=horizon, Minibatch=M, MinibatchGlobal=M_global,
                    Epochs=args.epochs, RandomizeStart=1, RandomizeMaterial=int(materials),
                    LanesPerWalker=args.lanes, RoughFloor=int(rough))
    try:
        if physics_only:
            import numpy as np
            g = torch.Generator(device="cuda").manual_seed(args.seed)
            acts = torch.rand((horizon, n, 4), device="cuda", generator=g) * 2 - 1
            rew = torch.empty((horizon, n), device="cuda")
            done = torch.empty((horizon, n), device="cuda", dtype=torch.uint8)
            torch.cuda.synchronize()
            step = lambda: eng.step_device(acts.data_ptr(), horizon, None, rew.data_ptr(),
                                           done.data_ptr(), None)
            eng.snapshot()
            time_iterations(eng, args, 2, horizon, 0, physics_only=step)  # warm-up
            reps = 16
            eng.profile_reset()
            eng.profile_enable(1)
            dt = time_iterations(eng, args, reps, horizon, 0, physics_only=step)
            prof = eng.profile()
            eng.profile_enable(0)
            launch_ms = prof["physics_ms"] / max(1, prof["physics_launches"])
            # the counting replay reads the trajectory buffer's actions: the same uniform
            # actions every timed launch stepped with, from the same restored state
            z = lambda *sh: np.zeros(sh, np.float32)
            eng.set_trajectory(z(horizon, n, 12), acts.cpu().numpy(), z(horizon, n, 4),
                               z(horizon, n), np.zeros((horizon, n), np.uint8), z(horizon, n))
            return {"walkers": n, "env_steps_timed": reps * n * horizon,
                    "env_steps_per_s": reps * n * horizon / dt,
                    "physics_ms_per_launch": launch_ms,
                    "roofline": rollout_roofline(eng, wk, launch_ms, n * horizon, horizon,
                                                 policy=False)}
        for it in range(args.regime_iters):
            eng.rollout(horizon)
            eng.ppo_update(update_index=it, sync=False)
        eng.snapshot()
        time_iterations(eng, args, 1, horizon, args.regime_iters)
        eng.profile_reset()
        eng.profile_enable(1)
        dt = time_iterations(eng, args, k, horizon, args.regime_iters)
        prof = eng.profile()
        eng.profile_enable(0)
        eng.profile_reset()
        eng.profile_enable(2)  # untimed: an event pair around every launch of one iteration
        time_iterations(eng, args, 1, horizon, args.regime_iters)
        eng.profile_enable(0)
        prof_k = eng.profile()
        upd_ms = prof["update_ms"] / max(1, prof["update_calls"])
        burst = eng.time_gradient(M, GRAD_BURST)
        burst_ev = eng.time_gradient(M, GRAD_BURST, per_launch_events=True)
        launch_ms = prof["physics_ms"] / max(1, prof["physics_launches"])
        return {"walkers": n, "minibatch": M, "minibatch_global": M_global,
                "env_steps_per_s": k * n * horizon / dt,
                "rollout_ms": launch_ms,
                "rollout_env_steps_per_s": n * horizon / max(1e-12, launch_ms * 1e-3),
                "ppo_update_ms": upd_ms,
                "minibatches_per_update": args.epochs * (n * horizon // M),
                "roofline": rollout_roofline(eng, wk, launch_ms, n * horizon, horizon),
                "roofline_update": update_roofline(prof_k, M, n, horizon, args.epochs, upd_ms, burst,
                                                   burst_ev, eng.grad_kernel(M))}
    finally:
        eng.close()


LINE_LIMIT = 4096  # the driver parses one stdout line; round 4's 20 KB line was lost


def _r(x, nd=4):
    """round a float to nd significant digits for the compact line (ints / None unchanged)"""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


def _trim_roofline(rf):
    keep = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "peak_no_fma",
            "frac_no_fma", "flop_per_env_step_counted", "mean_launch_ms", "hbm_GBs")
    out = {k: _r(rf[k]) for k in keep if k in rf}
    if "mapping" in rf:
        m = rf["mapping"]
        out["mapping"] = [m.get("lanes_per_walker"), m.get("walkers_per_wave"),
                          m.get("waves_launched", m.get("waves"))]
    return out


def _trim_update(ru):
    keep = ("kernel", "achieved", "peak", "unit", "frac", "mean_launch_us",
            "reduce_adam_us", "reduce_exchange_adam_us", "allreduce_us", "adam_us")
    out = {k: _r(ru[k]) for k in keep if k in ru}
    out["kernel"] = out.get("kernel", "").split(" ")[0]
    if "update" in ru:
        out["update_frac"] = _r(ru["update"]["frac"])
    return out


def compact_line(full, detail_file=None):
    """the <= 4 KB stdout line: the headline keys, config, the trimmed rollout and
    update rooflines, the CPU baseline's numbers and one summary per extra shape; everything
    else (event rates, notes, burst timings, the one-rank RCCL timing) stays in the detail file
    the line names"""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data")
    out = {k: full[k] for k in keys if k in full}
    cfg = dict(full.get("config", {}))
    xc = cfg.pop("exchange_check", None)
    if xc is not None:
        cfg["exchange_checked"] = bool(xc.get("checked")) and bool(xc.get("bitwise_equal_to_reference"))
    out["config"] = cfg
    for k in ("ppo_update_ms", "rollout_env_steps_per_s"):
        if k in full:
            out[k] = _r(full[k])
    if "regime" in full:
        out["regime"] = full["regime"]
    if "roofline" in full:
        out["roofline"] = _trim_roofline(full["roofline"])
    if "roofline_update" in full:
        out["roofline_update"] = _trim_update(full["roofline_update"])
    if "cpu_baseline" in full:
        c = full["cpu_baseline"]
        ac = c.get("all_cores", {})
        out["cpu_baseline"] = {
            "value": _r(c["value"]), "unit": c["unit"], "cores": c["cores"], "kind": c["kind"],
            "sample": c["sample"][:120],
            "physics_only": _r(c.get("physics_only_env_steps_per_s")),
            "train_ms": _r(c.get("train_ms_per_1001_step_episode")),
            "all_cores": {"threads": ac.get("threads"), "env_steps_per_s": _r(ac.get("env_steps_per_s")),
                          "cpu": ac.get("cpu_model")}}
    if "configs" in full:
        sm = {}
        for name, c in full["configs"].items():
            s = {"env_steps_per_s": _r(c.get("env_steps_per_s"))}
            if "rollout_ms" in c:
                s["rollout_ms"] = _r(c["rollout_ms"])
            if "physics_ms_per_launch" in c:
                s["physics_ms"] = _r(c["physics_ms_per_launch"])
            if "ppo_update_ms" in c:
                s["ppo_update_ms"] = _r(c["ppo_update_ms"])
            if "roofline" in c:
                s["frac"] = _r(c["roofline"]["frac"], 3)
            if "roofline_update" in c:
                s["update_frac"] = _r(c["roofline_update"]["frac"], 3)
            sm[name] = s
        out["configs"] = sm
    if "rehearsal" in full:
        out["rehearsal"] = full["rehearsal"]
    if full.get("xch_profile"):
        out["xch_profile_us"] = [None if r is None else
                                 {k: _r(r[k + "_us_median"], 3) for k in ("span", "wait", "own", "gap")}
                                 for r in full["xch_profile"]["per_rank"]]
    if detail_file:
        out["detail_file"] = detail_file
    line = json.dumps(out, separators=(",", ":"))
    if len(line) >= LINE_LIMIT:  # never lose the headline: drop the optional parts first
        for k in ("configs", "xch_profile_us", "regime", "rollout_env_steps_per_s", "cpu_baseline",
                  "roofline_update", "config"):
            out.pop(k, None)
            line = json.dumps(out, separators=(",", ":"))
            if len(line) < LINE_LIMIT:
                break
    if len(line) >= LINE_LIMIT:  #  the contract keys alone + where the rest went
        out = {k: out[k] for k in keys + ("detail_file",) if k in out}
        for k in ("metric", "data"):
            if isinstance(out.get(k), str):
                out[k] = out[k][:400]
        line = json.dumps(out, separators=(",", ":"))
    return line


def write_detail(full, path):
    """the full result (every roofline field, event rates, notes) as indented JSON; returns the
    repo-relative path named in the line, or None if it cannot be written"""
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
    except OSError as ex:
        print(f"bench: detail file not written ({ex})", file=sys.stderr)
        return None
    return os.path.relpath(path, ROOT)


def _claim_stdout():
    """the driver reads stdout for ONE JSON line; libraries print to fd 1 on their own (RCCL's
    version banner at the first collective), so fd 1 goes to stderr for the whole run and the
    JSON line is written to the original stdout"""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def allreduce_one_rank(wk, eng, args, horizon, update_index):
    """the collective path on one GPU -- a one-rank RCCL communicator makes
    wk_ppo_update run ordered reduction -> ncclAllReduce (24.6 KB, on the engine stream) ->
    Adam per minibatch, as every rank of the multi-GPU run does; one untimed profiled
    iteration gives the mean RCCL call time (a one-rank all-reduce moves no data over xGMI:
    a lower bound on the N > 1 exchange's latency)"""
    eng.comm_init(0, 1, wk.Engine.comm_unique_id())
    eng.profile_reset()
    eng.profile_enable(2)
    time_iterations(eng, args, 2, horizon, update_index)
    eng.profile_enable(0)
    p = eng.profile()
    calls = max(1, p["allreduce_calls"])
    return {"bytes": SLAB_BYTES, "calls": p["allreduce_calls"],
            "ms_per_call": p["allreduce_ms"] / calls,
            "ms_per_update": p["allreduce_ms"] / 2, "update_ms": p["update_ms"] / 2,
            "kernel_ms_one_step": {k: v / 2 for k, v in p.items() if k.endswith("_ms")},
            "note": "one-rank RCCL communicator on this GPU: the collective path of every rank"}


def ipc_exchange_setup(wk, eng, mk_engine, rank, world, horizon, dist, torch, np, rehearse=False):
    """N > 1 with --exchange ipc: map the peers' exchange regions (every rank joins
    the record all-gather, also when its own handle failed), run one test round on exact small
    integers, vote; then check the one-shot exchange against an EXACT reference over several
    updates: a second context on the same shard whose host exchange all-gathers the slabs over
    gloo and sums them in rank order in float32 (the IPC kernel's association, so the result is
    bit-identical whatever N) -- two PPO iterations of 2 epochs each from the seeded start, then
    the weights, Adam moments and walker records compared bit for bit, and the replicas'
    weights compared across ranks.  Any failure returns 0 (bench.py then falls back to RCCL on
    every rank).  The IPC context is restored to its seeded start afterwards."""
    def allgather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    def vote(ok):
        t = torch.tensor([int(ok)])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    check = {"test_round": False, "checked": False}
    ok = True
    # rehearsal-only fault injection: this rank reports a wrong test-round sum,
    # so every rank must take the fallback exchange and still print exactly one line
    fault_rank = int(os.environ.get("WK_BENCH_FAULT_RANK", "-1")) if rehearse else -1
    try:
        eng.comm_init_ipc(rank, world, allgather)
        check["region"] = "uncached device memory" if eng.comm_info()[1] else "hipMalloc"
        base = (np.arange(wk.NPARAM) % 97).astype(np.float32)
        got = eng.allreduce_test(base + np.float32(rank + 1))
        if rank == fault_rank:
            got = got + np.float32(1)
        want = base * np.float32(world) + np.float32(world * (world + 1) // 2)
        ok = bool(np.array_equal(got, want))
        if not ok:
            print(f"rank {rank}: IPC exchange test gave wrong sums", file=sys.stderr)
    except wk.WkError as ex:  # e.g. no peer access between the devices, a peer timed out
        print(f"rank {rank}: IPC exchange unavailable ({ex})", file=sys.stderr)
        ok = False
    if not vote(ok):
        return 0, check
    check["test_round"] = True

    def rank_order_sum(buf):
        t = torch.from_numpy(buf.copy())
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        acc = parts[0].numpy().copy()
        for p in parts[1:]:
            acc = acc + p.numpy()  # float32, rank order
        buf[:] = acc

    ref = mk_engine()
    updates, epochs = 2, 2
    same, t, wbytes = False, 0, b""
    try:
        ref.comm_init_host(rank, world, rank_order_sum)
        eng.snapshot()
        for u in range(updates):
            for e in (eng, ref):
                e.rollout(horizon)
                e.ppo_update(epochs=epochs, update_index=1000 + u)
        w, (m, v, t) = eng.get_weights(), eng.get_adam()
        same = (np.array_equal(w, ref.get_weights()) and np.array_equal(m, ref.get_adam()[0])
                and np.array_equal(v, ref.get_adam()[1]) and t == ref.get_adam()[2]
                and np.array_equal(eng.get_state(), ref.get_state()))
        wbytes = w.tobytes()
        eng.restore()
    except wk.WkError as ex:
        print(f"rank {rank}: IPC exchange check failed ({ex})", file=sys.stderr)
        same, t, wbytes = False, 0, b""
    finally:
        ref.close()
    # every rank joins the replica all-gather, also after a failure: a rank that
    # skipped it would pair its peers' all_gather_object with main's vote and hang the job
    replicas = allgather(wbytes)
    identical = bool(wbytes) and all(r == replicas[0] for r in replicas)
    check.update({"checked": True, "updates": updates, "epochs_per_update": epochs,
                  "adam_steps": int(t), "bitwise_equal_to_reference": bool(same),
                  "replicas_identical": bool(identical),
                  "reference": "rank-order float32 sum of the ranks' slabs all-gathered over gloo"})
    if not (same and identical):
        print(f"rank {rank}: IPC exchange differs from the rank-order reference", file=sys.stderr)
    return int(same and identical), check


def xch_stamp_summary(st):
    """per-minibatch split of the IPC exchange kernel (k_reduce_xch_adam) from its per-block
    constant-clock stamps [launch, block, (entry, published, peers seen, exit)], 10 ns ticks:
    span = last exit - first entry of the launch; wait = a block's (peers seen - published);
    own = (published - entry) + (exit - peers seen), the block's reduction, publish, peer reads and
    Adam; gap = next launch's first entry - this launch's last exit (the gradient kernel between)"""
    import numpy as np
    if len(st) == 0:
        return None
    st = st.astype(np.float64) * 0.01  # ticks of the 100 MHz clock -> microseconds
    span = st[:, :, 3].max(axis=1) - st[:, :, 0].min(axis=1)
    wait = st[:, :, 2] - st[:, :, 1]
    own = (st[:, :, 1] - st[:, :, 0]) + (st[:, :, 3] - st[:, :, 2])
    gap = st[1:, :, 0].min(axis=1) - st[:-1, :, 3].max(axis=1)
    med = lambda a: float(np.median(a)) if a.size else None
    return {"launches": int(st.shape[0]), "blocks": int(st.shape[1]),
            "span_us_median": med(span), "span_us_mean": float(span.mean()),
            "wait_us_median": med(np.median(wait, axis=1)), "wait_us_max_median": med(wait.max(axis=1)),
            "own_us_median": med(np.median(own, axis=1)), "own_us_max_median": med(own.max(axis=1)),
            "gap_us_median": med(gap)}


def main():
    args = parse()
    json_out = _claim_stdout()
    import wk
    from wk.dist import broadcast_unique_id, env_from_launcher, make_shard

    rank, world, local = env_from_launcher()
    if world != args.gpus and world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    # the CPU leg first, before this process touches the GPU (its workers are spawned)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    import numpy as np
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; gradients go over RCCL
    if args.rehearse:
        local = 0
    elif torch.cuda.device_count() == 1 and local > 0:
        local = 0  # a launcher that shows each rank only its own GPU (HIP_VISIBLE_DEVICES)
    torch.cuda.set_device(local)
    weak = args.walkers > 0
    if weak:
        n_local = args.walkers
        m_global = args.minibatch_global or n_local * world
    else:
        if args.walkers_global % world:
            raise SystemExit("--walkers-global must divide by the number of GPUs")
        n_local = args.walkers_global // world
        m_global = args.minibatch_global or args.walkers_global
    if m_global % world:
        raise SystemExit("the global minibatch must divide by the number of GPUs")
    shard = make_shard(rank, world, local, n_local, m_global // world)
    T = args.horizon
    mk_engine = lambda: wk.Engine(
        shard.n_local, seed=args.seed, device=local, Horizon=T, Minibatch=shard.minibatch_local,
        MinibatchGlobal=shard.minibatch_global, Epochs=args.epochs, EnvOffset=shard.env_offset,
        RandomizeStart=1, RandomizeMaterial=1 if args.materials else 0, LanesPerWalker=args.lanes)
    eng = mk_engine()
    exchange = args.exchange if world > 1 else "none"
    xch_check = None
    if world > 1 and args.exchange == "ipc":
        ok, xch_check = ipc_exchange_setup(wk, eng, mk_engine, rank, world, T, dist, torch, np,
                                           rehearse=args.rehearse)
        okt = torch.tensor([ok])
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)  # every rank takes the same exchange
        if not okt.item():
            eng.close()
            eng = mk_engine()
            exchange = "host (gloo)" if args.rehearse else "rccl"
    if world > 1 and exchange != "ipc" and args.rehearse:
        def host_allreduce(buf):
            t = torch.from_numpy(buf)
            dist.all_reduce(t)  # in place on the numpy view (gloo)
        eng.comm_init_host(rank, world, host_allreduce)
        exchange = "host (gloo)"
    elif world > 1 and exchange != "ipc":
        uid = wk.Engine.comm_unique_id() if rank == 0 else None
        uid = broadcast_unique_id(uid)
        eng.comm_init(rank, world, uid)
        exchange = "rccl"

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # fixed regime: R iterations from the seeded start, then the device snapshot
    for it in range(args.regime_iters):
        eng.rollout(T)
        eng.ppo_update(update_index=it, sync=False)
    eng.snapshot()
    upd = args.regime_iters
    time_iterations(eng, args, args.warmup, T, upd, barrier)
    eng.profile_reset()
    eng.profile_enable(1)  # one HIP event pair per rollout launch and per whole update
    elapsed = time_iterations(eng, args, args.steps, T, upd, barrier)
    prof = eng.profile()
    eng.profile_enable(0)
    # untimed: one iteration with an event pair around every kernel launch
    eng.profile_reset()
    eng.profile_enable(2)
    time_iterations(eng, args, 1, T, upd)
    eng.profile_enable(0)
    prof_k = eng.profile()
    # untimed: the gradient kernel alone, back to back, timed by one event pair and by a pair
    # around every launch (their difference: the per-launch event overhead, subtracted from the
    # level-2 in-update mean for the update roofline)
    grad_burst_ms = eng.time_gradient(shard.minibatch_local, GRAD_BURST)
    grad_burst_ev_ms = eng.time_gradient(shard.minibatch_local, GRAD_BURST, per_launch_events=True)
    # untimed: one iteration with the exchange kernel's per-block clock stamps
    xch_prof = None
    if args.xch_profile and exchange == "ipc":
        n_mb = args.epochs * (shard.n_local * T // shard.minibatch_local)
        eng.xch_profile(n_mb)
        time_iterations(eng, args, 1, T, upd, barrier)
        mine = xch_stamp_summary(eng.xch_stamps(n_mb))
        eng.xch_profile(0)
        xch_prof = [None] * world
        dist.all_gather_object(xch_prof, mine)
    # untimed: the timed iteration's episode count, then its physics events (counting replay of
    # its actions from the restored state) for the rollout roofline
    eng.restore()
    eng.rollout(T)
    stats = eng.rollout_stats()

    t = torch.tensor([elapsed, prof["physics_ms"], prof["update_ms"]], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, phys_ms_max, upd_ms_max = t.tolist()

    env_steps = world * shard.n_local * T * args.steps
    value = env_steps / elapsed
    launch_ms = prof["physics_ms"] / max(1, prof["physics_launches"])
    units = prof["physics_env_steps"] / max(1, prof["physics_launches"])
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            tj = json.load(open(args.traffic_file))
            if tj.get("walkers") == shard.n_local and tj.get("horizon") == T:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    roofline = rollout_roofline(eng, wk, launch_ms, units, T, traffic=traffic)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox-randomised start offsets; random-init Xavier policy)",
        "config": {
            "workload": (f"BASELINE config 4: {shard.n_local * world} walkers over {world} GPU(s) "
                         f"({shard.n_local}/GPU), config 3 step: rollout T_h={T} with policy "
                         f"sampling + PPO update E={args.epochs}, global minibatch "
                         f"{shard.minibatch_global} ({shard.minibatch_local}/GPU)"
                         + (", per-env Ice/Rubber/Carpet (config 5)" if args.materials else "")),
            "walkers_per_gpu": shard.n_local,
            "global_walkers": shard.n_local * world,
            "horizon": T,
            "epochs": args.epochs,
            "minibatch_global": shard.minibatch_global,
            "parallelism": f"dp{world}",
            "exchange": exchange,
        },
        "ppo_update_ms": upd_ms_max / args.steps,
        "rollout_env_steps_per_s": world * shard.n_local * T * args.steps / (phys_ms_max * 1e-3),
        "regime": {"iterations_before_snapshot": args.regime_iters,
                   "episodes_per_rollout": int(stats.episodes)},
        "roofline": roofline,
        "kernel_ms_one_step": {k: v for k, v in prof_k.items() if k.endswith("_ms")},
        "roofline_update": update_roofline(prof_k, shard.minibatch_local, shard.n_local, T,
                                           args.epochs, upd_ms_max / args.steps, grad_burst_ms,
                                           grad_burst_ev_ms, eng.grad_kernel(shard.minibatch_local),
                                           exchange),
    }
    if xch_check is not None:
        out["config"]["exchange_check"] = xch_check
    if xch_prof is not None:
        out["xch_profile"] = {"per_rank": xch_prof, "note": xch_stamp_summary.__doc__.split(";")[0]}
    if world == 1 and not args.rehearse:
        out["allreduce_1rank"] = allreduce_one_rank(wk, eng, args, T, upd)
    if rank == 0 and world == 1 and not args.no_extras:
        ex = {}
        ex["config2_physics_4096"] = extra_config(wk, torch, args, 4096, 4096, 4096, T,
                                                  physics_only=True)
        ex["config3_full_4096"] = extra_config(wk, torch, args, 4096, 4096, 4096, T)
        ex["config4_shard_8192"] = extra_config(wk, torch, args, 8192, 8192, 65536, T)
        ex["config5_shard_8192"] = extra_config(wk, torch, args, 8192, 8192, 65536, T,
                                                materials=True)
        #  config 5 at its stated size: 65,536 walkers with per-env materials
        ex["config5_materials_65536"] = extra_config(wk, torch, args, 65536, 65536, 65536, T,
                                                     materials=True)
        ex["rough_floor_65536"] = extra_config(wk, torch, args, 65536, 65536, 65536, T, rough=True)
        ex["rough_floor_shard_8192"] = extra_config(wk, torch, args, 8192, 8192, 65536, T,
                                                    rough=True)
        out["configs"] = ex
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if args.rehearse:
        out["rehearsal"] = (f"all ranks on one GPU, exchange {exchange}: a check of the "
                            "multi-rank path, not a performance number")
    if rank == 0:
        detail = write_detail(out, args.detail_file) if args.detail_file else None
        print(compact_line(out, detail), file=json_out, flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
