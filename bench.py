#!/usr/bin/env python3
"""bench.py -- batched bipedal-walker physics + PPO on MI355X (BASELINE.json metric).

One "step" = one PPO iteration over this rank's walkers: a device-resident rollout of
`--horizon` env-steps (policy sampling + 50 physics substeps + reward/terminal/auto-reset
+ value estimate, fused in one HIP kernel) followed by the returns scan and the PPO
update (E epochs x pool/M minibatches: gradient kernel -> ordered reduction -> RCCL
all-reduce -> Adam).  The metric's configuration (BASELINE.json: 65,536 walkers) fits one MI355X, so it is the
N=1 workload; walkers are independent, so N GPUs run weakly scaled shards of --walkers
each (65,536 per GPU) with only the policy-gradient all-reduce between them.
value = env-steps of all ranks / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W --walkers 8192 --horizon 64]
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
# algorithmic fp32 flops per env-step (50 substeps x 5,775 + actor
# forward 10,504 + sampling/log-prob/obs/reward ~130) and bytes per env-step.
FLOP_PER_ENV_STEP = 3.0e5
BYTES_PER_ENV_STEP = 950.0
PEAK_FP32_TFLOPS = 157.3   # MI355X fp32 vector (= fp32 matrix) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--walkers", type=int, default=65536, help="walkers per GPU")
    p.add_argument("--horizon", type=int, default=64)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--minibatch", type=int, default=0, help="per-GPU minibatch (0 = walkers)")
    p.add_argument("--materials", action="store_true", help="config 5: random Ice/Rubber/Carpet")
    p.add_argument("--seed", type=int, default=20250905)
    p.add_argument("--lanes", type=int, default=0,
                   help="lanes per walker in the physics kernel (0 auto, 1, 2 or 16)")
    p.add_argument("--cpu-baseline-steps", type=int, default=150000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_physics.json"))
    return p.parse_args()


def cpu_baseline(args):
    """The oracle's single-walker reference loop (Game1.Update -> Environment.Update with
    Train at every terminal step, 5 epochs x floor(T/64) x 64), on one host core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    orc.build()
    n = args.cpu_baseline_steps
    t0 = time.perf_counter()
    eps, train_s = orc.reference_loop(n, seed=args.seed)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{n} env-steps of the single-walker reference loop (policy + physics, "
                      f"PPO Train at each of {eps} episode ends: {train_s:.2f} s of {dt:.2f} s)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import wk
    from wk.dist import broadcast_unique_id, env_from_launcher, make_shard

    rank, world, local = env_from_launcher()
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; gradients go over RCCL
    torch.cuda.set_device(local)
    shard = make_shard(rank, world, local, args.walkers, args.minibatch or args.walkers)
    eng = wk.Engine(shard.n_local, seed=args.seed, device=local, Horizon=args.horizon,
                    Minibatch=shard.minibatch_local, MinibatchGlobal=shard.minibatch_global,
                    Epochs=args.epochs, EnvOffset=shard.env_offset, RandomizeStart=1,
                    RandomizeMaterial=1 if args.materials else 0, LanesPerWalker=args.lanes)
    if world > 1:
        uid = wk.Engine.comm_unique_id() if rank == 0 else None
        uid = broadcast_unique_id(uid)
        eng.comm_init(rank, world, uid)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    it = 0
    for _ in range(args.warmup):
        eng.rollout(args.horizon)
        eng.ppo_update(update_index=it, sync=False)
        it += 1
    barrier()
    eng.profile_reset()
    eng.profile_enable(1)  # one HIP event pair per rollout launch and per whole update
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.rollout(args.horizon)
        eng.ppo_update(update_index=it, sync=False)
        it += 1
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = eng.profile()
    stats = eng.rollout_stats()
    # one more (untimed) iteration with an event pair around every kernel launch
    eng.profile_reset()
    eng.profile_enable(2)
    eng.rollout(args.horizon)
    eng.ppo_update(update_index=it, sync=False)
    eng.sync()
    eng.profile_enable(0)
    prof_k = eng.profile()

    t = torch.tensor([elapsed, prof["physics_ms"], prof["update_ms"] + prof["returns_ms"]],
                     dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, phys_ms_max, upd_ms_max = t.tolist()

    env_steps = world * shard.n_local * args.horizon * args.steps
    value = env_steps / elapsed
    phys_launch_ms = prof["physics_ms"] / max(1, prof["physics_launches"])
    units_per_launch = prof["physics_env_steps"] / max(1, prof["physics_launches"])
    achieved_tflops = FLOP_PER_ENV_STEP * units_per_launch / (phys_launch_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            tj = json.load(open(args.traffic_file))
            if tj.get("walkers") == shard.n_local and tj.get("horizon") == args.horizon:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    ppo_update_ms = upd_ms_max / args.steps
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox-randomised start offsets; random-init Xavier policy)",
        "config": {
            "workload": ("BASELINE config 4 walker count (65,536) per GPU, config 3 step: "
                         f"{shard.n_local} walkers/GPU, rollout T_h={args.horizon} with policy "
                         f"sampling + PPO update E={args.epochs}, M={shard.minibatch_local}/GPU"
                         + (", per-env Ice/Rubber/Carpet (config 5)" if args.materials else "")),
            "walkers_per_gpu": shard.n_local,
            "global_walkers": shard.n_local * world,
            "horizon": args.horizon,
            "epochs": args.epochs,
            "minibatch_global": shard.minibatch_global,
            "parallelism": f"dp{world}",
        },
        "ppo_update_ms": ppo_update_ms,
        "rollout_env_steps_per_s": world * shard.n_local * args.horizon * args.steps / (phys_ms_max * 1e-3),
        "roofline": {
            "bound": "mfma",
            "kernel": {2: "k_env_side<true,true,false>", 16: "k_env_step<true,true,false,16>",
                       1: "k_env_step<true,true,false,1>"}[args.lanes or (2 if shard.n_local >= 32768 else 16)]
                      + " (fused rollout: physics + policy)",
            "achieved": achieved_tflops,
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tflops / PEAK_FP32_TFLOPS,
            "traffic": traffic,
            "note": ("fp32 compute-bound (VALU; the MI355X fp32 vector peak equals the fp32 "
                     "MFMA peak, 157.3 TF); algorithmic flops = 3.0e5 per env-step (SURVEY 8(d)) "
                     f"x {units_per_launch:.0f} env-steps per launch / {phys_launch_ms:.3f} ms "
                     "mean launch (HIP events on the engine stream)"),
            "hbm_frac": BYTES_PER_ENV_STEP * units_per_launch / (phys_launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
        },
        "kernel_ms_one_step": {k: v for k, v in prof_k.items() if k.endswith("_ms")},
        "episodes_last_rollout": stats.episodes,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
