"""GPU parity: libwk.so (HIP, gfx950) against the CPU oracle, through the C ABI.

Bars (SURVEY.md 8 / BASELINE north_star):
  * physics with given actions: bit-exact -- AABB/SAT/contact bookkeeping per substep,
    body poses / velocities / flags after 1 and 1000 env-steps (drift 0 < 1e-4);
  * policy forward / sampling: fp32 within rtol 1e-5 (device libm transcendentals
    differ from glibc by <= 1-2 ulp), the same Philox noise;
  * Train(Batch): gradient within rtol 1e-4 / atol 1e-7 (sample accumulation order),
    Adam-updated weights within atol 1e-6.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905
F = np.float32
LANES = [1, 2, 4, 16]  # physics mappings: lane per walker, side-split pair, split leg pairs, SAT rows
lanes_param = pytest.mark.parametrize("lanes", LANES)


def oracle_envs(orc, eng, n):
    dx = [orc.env_offset(SEED, e) for e in range(n)]
    mats = [orc.env_material(SEED, e) for e in range(n)]
    return [orc.Env(dx=float(dx[e]), material=int(mats[e])) for e in range(n)], dx, mats


@pytest.fixture(scope="module")
def eng64(wk):
    e = wk.Engine(64, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Horizon=32)
    yield e
    e.close()


def test_template_state_bitexact(wk, orc):
    n = 256
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    envs, _, _ = oracle_envs(orc, eng, n)
    ref = np.stack([e.dump() for e in envs])
    np.testing.assert_array_equal(eng.get_state(), ref)
    np.testing.assert_array_equal(eng.get_obs(), np.stack([e.obs() for e in envs]))


@lanes_param
def test_one_step_trace_bitexact(wk, orc, lanes):
    n = 128
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, LanesPerWalker=lanes)
    envs, _, _ = oracle_envs(orc, eng, n)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1.3, 1.3, (n, 4)).astype(F)  # includes clipped values
    tr = eng.step_traced(acts)
    for i, e in enumerate(envs):
        _, _, _, t = e.step(acts[i], trace=True)
        for k in ("aabb_hit", "sat_hit", "n_contacts"):
            np.testing.assert_array_equal(tr[i][k], t[k], err_msg=f"env {i} {k}")
        for k in ("normal", "depth", "contact", "impulse", "joint_depth", "joint_impulse"):
            np.testing.assert_array_equal(tr[i][k], t[k], err_msg=f"env {i} {k}")
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))


@lanes_param
def test_golden_one_step(wk, golden, lanes):
    g = golden("env_step_trace.npz")
    eng = wk.Engine(1, seed=SEED, LanesPerWalker=lanes)
    np.testing.assert_array_equal(eng.get_state()[0], g["state0"])
    tr = eng.step_traced(g["action"][None])[0]
    for k in ("aabb_hit", "sat_hit", "n_contacts", "normal", "depth"):
        np.testing.assert_array_equal(tr[k], g[k])
    np.testing.assert_array_equal(eng.get_state()[0], g["state1"])


@lanes_param
def test_golden_thousand_steps_bitexact(wk, orc, golden, lanes):
    """1000 identical env-steps for 8 walkers (auto-resets included): drift must be 0."""
    g = golden("thousand_steps.npz")
    n = g["dx"].size
    eng = wk.Engine(n, seed=SEED, LanesPerWalker=lanes)
    eng.set_offsets(g["dx"])
    eng.reset()
    # the fixture starts in episode 0 (floor last): restore that flag after the reset
    st = eng.get_state()
    st[:, 109] = 0
    eng.set_state(st)
    acts = np.stack([[orc.synth_action(SEED, i, t) for i in range(n)] for t in range(1000)])
    for blk in range(10):
        obs, rew, done, fault = eng.step(acts[blk * 100:(blk + 1) * 100], k=100)
        np.testing.assert_array_equal(rew, g["rewards"][blk * 100:(blk + 1) * 100])
        np.testing.assert_array_equal(done, g["dones"][blk * 100:(blk + 1) * 100])
        np.testing.assert_array_equal(eng.get_state(), g["snaps"][blk], err_msg=f"block {blk}")
        assert not fault.any()


@lanes_param
def test_many_envs_multi_step_bitexact(wk, orc, lanes):
    n, k = 512, 40
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, LanesPerWalker=lanes)
    envs, _, _ = oracle_envs(orc, eng, n)
    rng = np.random.default_rng(5)
    acts = rng.uniform(-1, 1, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
            np.testing.assert_array_equal(o, obs[t, i])
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))


@lanes_param
def test_reset_mask_and_materials(wk, orc, lanes):
    n = 16
    eng = wk.Engine(n, seed=SEED, LanesPerWalker=lanes)
    mats = np.array([0, 1, 2] * 5 + [0], np.int32)
    eng.set_materials(mats)
    acts = np.random.default_rng(2).uniform(-1, 1, (20, n, 4)).astype(F)
    eng.step(acts, k=20)
    mask = np.zeros(n, np.uint8)
    mask[::2] = 1
    eng.reset(mask)
    envs = [orc.Env(material=int(m)) for m in mats]
    for i, e in enumerate(envs):
        for t in range(20):
            e.step(acts[t, i])
        if mask[i]:
            e.reset()
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    bv = eng.body_view(3, 2)
    assert bv.n_vertices == 5 and eng.body_view(3, 5).is_static == 1


def test_policy_sample_matches_oracle(wk, orc, eng64):
    ag = orc.Agent(seed=SEED)
    np.testing.assert_allclose(eng64.get_weights(), ag.params(), rtol=0, atol=2e-7)
    eng64.set_weights(ag.params())
    rng = np.random.default_rng(3)
    obs = rng.normal(0, 1, (64, 12)).astype(F)
    ids = np.arange(64, dtype=np.int32)
    steps = np.full(64, 7, np.uint32)
    mean, act, lp = eng64.policy_sample(obs, ids, steps)
    for i in range(64):
        np.testing.assert_allclose(mean[i], ag.mean(obs[i]), rtol=1e-5, atol=1e-6)
        a, l = ag.sample(obs[i], SEED, i, 7)
        np.testing.assert_allclose(act[i], a, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(lp[i], l, rtol=1e-5, atol=1e-4)
    v = eng64.value(obs)
    np.testing.assert_allclose(v, [ag.value(o) for o in obs], rtol=1e-5, atol=1e-6)


@lanes_param
def test_rollout_physics_replays_exactly(wk, orc, lanes):
    """Policy rollout on the GPU; the oracle replays the recorded (unclipped) actions and
    must reproduce states, rewards and dones bit-exactly; the recorded actions match the
    oracle's own sampling within fp32 tolerance."""
    eng64 = wk.Engine(64, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Horizon=32,
                      LanesPerWalker=lanes)
    ag = orc.Agent(seed=SEED)
    eng64.set_weights(ag.params())
    eng64.reset()
    st = eng64.get_state()
    st[:, 109] = 0
    eng64.set_state(st)
    n, T = 64, 32
    envs, _, _ = oracle_envs(orc, eng64, n)
    step0 = 0  # per-env step counters may have advanced; read them back from the noise
    eng64.rollout(T)
    tr = eng64.get_trajectory(T)
    for i, e in enumerate(envs):
        for t in range(T):
            np.testing.assert_array_equal(tr["states"][t, i], e.obs(), err_msg=f"env {i} t {t}")
            o, r, d = e.step(tr["actions"][t, i])
            assert r == tr["rewards"][t, i] and d == tr["dones"][t, i]
    np.testing.assert_array_equal(eng64.get_state(), np.stack([e.dump() for e in envs]))
    v = np.array([[ag.value(tr["states"][t, i]) for i in range(n)] for t in range(T)], F)
    np.testing.assert_allclose(tr["values"], v, rtol=1e-5, atol=1e-6)
    _ = step0
    for i in range(n):
        ret, adv = orc.returns_mc(tr["rewards"][:, i], tr["values"][:, i], tr["dones"][:, i], 0.9)
        np.testing.assert_array_equal(tr["returns"][:, i], ret)
        np.testing.assert_array_equal(tr["advantages"][:, i], adv)


@lanes_param
def test_rollout_sampling_matches_oracle(wk, orc, lanes):
    ag = orc.Agent(seed=SEED)
    n, T = 32, 4
    eng = wk.Engine(n, seed=SEED, Horizon=T, LanesPerWalker=lanes)
    eng.set_weights(ag.params())
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    for i in range(n):
        for t in range(T):
            a, l = ag.sample(tr["states"][t, i], SEED, i, t)
            np.testing.assert_allclose(tr["actions"][t, i], a, rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(tr["logp"][t, i], l, rtol=1e-5, atol=1e-4)


def test_train_batch_matches_oracle(wk, orc, golden):
    g = golden("train_batch.npz")
    eng = wk.Engine(4, seed=SEED)
    eng.set_weights(g["w0"])
    eng.set_adam(np.zeros(wk.NPARAM), np.zeros(wk.NPARAM), 0)
    grads, cd, ad, sk = eng.train_batch(g["states"], g["actions"], g["logp_old"], g["returns"],
                                        g["adv"])
    np.testing.assert_allclose(grads, g["grads"], rtol=1e-4, atol=1e-7)
    assert sk == g["skipped"]
    assert cd == pytest.approx(float(g["critic_diag"]), rel=1e-4, abs=1e-7)
    assert ad == pytest.approx(float(g["actor_diag"]), rel=1e-4, abs=1e-7)
    np.testing.assert_allclose(eng.get_weights(), g["w1"], rtol=0, atol=2e-6)
    m, v, t = eng.get_adam()
    assert t == 1


def test_ppo_update_matches_oracle(wk, orc):
    """A whole PPO update (E epochs x pool/M minibatches, permuted sampling, Adam after
    each minibatch) against the oracle running the same minibatch sequence."""
    n, T, M, E = 16, 8, 32, 2
    eng = wk.Engine(n, seed=SEED, Horizon=T, Minibatch=M, Epochs=E)
    ag = orc.Agent(seed=SEED)
    eng.set_weights(ag.params())
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    cd, ad = eng.ppo_update(update_index=3)
    pool = n * T
    S = tr["states"].reshape(pool, 12)
    A = tr["actions"].reshape(pool, 4)
    L = tr["logp"].reshape(pool, 4)
    G = tr["returns"].reshape(pool)
    Ad = tr["advantages"].reshape(pool)
    for e in range(E):
        key = orc.perm_key(SEED, 3, e)
        for j in range(pool // M):
            idx = [orc.perm(j * M + k, pool, key) for k in range(M)]
            _, ocd, oad, _ = ag.train_batch(S[idx], A[idx], L[idx], G[idx], Ad[idx], b_div=M)
    np.testing.assert_allclose(eng.get_weights(), ag.params(), rtol=0, atol=5e-6)
    assert cd == pytest.approx(ocd, rel=1e-3, abs=1e-6)
    assert ad == pytest.approx(oad, rel=1e-3, abs=1e-6)
    m, v, t = eng.get_adam()
    assert t == E * (pool // M)


def test_gae_and_normalize_path(wk, orc):
    n, T = 8, 16
    eng = wk.Engine(n, seed=SEED, Horizon=T, UseGAE=1, NormalizeAdvantages=1)
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    adv = np.zeros((T, n), F)
    for i in range(n):
        ret, a = orc.returns_gae(tr["rewards"][:, i], tr["values"][:, i], tr["dones"][:, i], 0.9, 0.95)
        np.testing.assert_array_equal(tr["returns"][:, i], ret)
        adv[:, i] = a
    np.testing.assert_allclose(tr["advantages"], orc.normalize(adv.reshape(-1), 0.3).reshape(T, n),
                               rtol=1e-5, atol=1e-6)


def test_deterministic_rerun(wk):
    def run():
        eng = wk.Engine(256, seed=11, Horizon=16, Minibatch=512, RandomizeStart=1)
        eng.rollout(16)
        eng.ppo_update()
        w = eng.get_weights()
        s = eng.get_state()
        eng.close()
        return w, s
    w1, s1 = run()
    w2, s2 = run()
    np.testing.assert_array_equal(w1, w2)
    np.testing.assert_array_equal(s1, s2)


def test_single_rank_comm(wk):
    eng = wk.Engine(4, seed=1)
    uid = wk.Engine.comm_unique_id()
    eng.comm_init(0, 1, uid)
    x = np.arange(100, dtype=F)
    np.testing.assert_array_equal(eng.allreduce_test(x), x)


def test_step_device_pointers(wk):
    torch = pytest.importorskip("torch")
    n, k = 64, 3
    eng = wk.Engine(n, seed=SEED)
    ref = wk.Engine(n, seed=SEED)
    acts = torch.rand(k, n, 4, device="cuda") * 2 - 1
    obs = torch.empty(k, n, 12, device="cuda")
    rew = torch.empty(k, n, device="cuda")
    done = torch.empty(k, n, dtype=torch.uint8, device="cuda")
    fault = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    eng.step_device(acts.data_ptr(), k, obs.data_ptr(), rew.data_ptr(), done.data_ptr(),
                    fault.data_ptr())
    eng.sync()
    o2, r2, d2, _ = ref.step(acts.cpu().numpy(), k=k)
    np.testing.assert_array_equal(obs.cpu().numpy(), o2)
    np.testing.assert_array_equal(rew.cpu().numpy(), r2)
    np.testing.assert_array_equal(done.cpu().numpy(), d2)


def test_mappings_agree_at_scale(wk):
    """Size-independent properties at the bench's per-GPU size (65,536 walkers): the
    three physics mappings step bit-identically on the same actions, and a policy
    rollout of the default (side-split, matrix-core policy) mapping replays exactly
    through the one-lane mapping's physics."""
    n, T = 65536, 4
    rng = np.random.default_rng(9)
    acts = rng.uniform(-1.2, 1.2, (T, n, 4)).astype(F)
    outs = []
    for lanes in LANES:
        eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RandomizeMaterial=1,
                        LanesPerWalker=lanes)
        obs, rew, done, fault = eng.step(acts, k=T)
        outs.append((eng.get_state(), obs, rew, done))
        eng.close()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)
    roll = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RandomizeMaterial=1,
                     LanesPerWalker=2)
    replay = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RandomizeMaterial=1,
                       LanesPerWalker=1)
    roll.rollout(T)
    tr = roll.get_trajectory(T)
    obs, rew, done, _ = replay.step(tr["actions"], k=T)
    np.testing.assert_array_equal(rew, tr["rewards"])
    np.testing.assert_array_equal(done, tr["dones"])
    np.testing.assert_array_equal(obs[:-1], tr["states"][1:])
    np.testing.assert_array_equal(replay.get_state(), roll.get_state())


def test_invalid_lanes_rejected(wk):
    with pytest.raises(wk.WkError):
        wk.Engine(4, seed=SEED, LanesPerWalker=3)


@pytest.mark.parametrize("B", [1, 37, 2048])
def test_minibatch_gradient_mfma_vs_oracle(wk, orc, B):
    """The matrix-core gradient (wk_ppo_update's kernel) against the oracle's sequential
    Train(Batch) on the same samples: fp32 re-association only (16-sample MFMA blocks,
    4-way split dots), so rtol 2e-4 / atol 2e-6 relative to the largest gradient."""
    rng = np.random.default_rng(B)
    ag = orc.Agent(seed=SEED)
    eng = wk.Engine(4, seed=SEED)
    eng.set_weights(ag.params())
    S = rng.normal(0, 1, (B, 12)).astype(F)
    A = rng.normal(0, 1, (B, 4)).astype(F)
    L = rng.normal(-3, 1, (B, 4)).astype(F)
    G = rng.normal(0, 5, B).astype(F)
    Ad = rng.normal(0, 1, B).astype(F)
    if B > 5:
        L[5, 2] = -200.0  # exp(logp_old) == 0: HadamardDivision throws, sample skipped
    g, cd, ad, sk = eng.minibatch_gradient(S, A, L, G, Ad)
    og, ocd, oad, osk = ag.train_batch(S, A, L, G, Ad, b_div=B, apply_adam=False)
    scale = np.abs(og).max()
    np.testing.assert_allclose(g, og, rtol=2e-4, atol=2e-6 * scale)
    assert sk == osk
    assert cd == pytest.approx(ocd, rel=1e-4, abs=1e-6)
    assert ad == pytest.approx(oad, rel=1e-4, abs=1e-6)


def test_fast_sqrt_rcp_exhaustive():
    """The physics kernel's sqrt_rn / rsqrt_rn / rcp_core equal HIP's correctly rounded
    sqrtf and division on every non-negative float (tests/cpp/fastmath_check.hip)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ppo-bipedalwalker_amd", "build", "fastmath_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe)), "check"],
                       check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout


def test_floor_face_closed_form():
    """The flat floor's contact face from the argmin index bits (floor_face_ax) equals the
    generic significant_face_ax over the floor polygon bit for bit, for 2^26 hashed normals
    and every pair of 24 special components (tests/cpp/floor_face_check.hip)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ppo-bipedalwalker_amd", "build", "floor_face_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe)), "check"],
                       check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


def test_row_exchanges_bit_identical():
    """The permlane / DPP lane-group exchanges (wk_mfma_layout.h rows_sum4 / rows_max4 /
    rows_bcast4 / rows_rsum4 / row_tree16) equal the __shfl / LDS formulations they replaced, bit
    for bit, on 67 M hashed floats incl. signed zeros and infinities (tests/cpp/rows_check.hip)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ppo-bipedalwalker_amd", "build", "rows_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe)), "check"],
                       check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


def test_baseline_config2_physics_4096(wk, orc):
    """BASELINE config 2: 4,096 walkers, physics-step only (auto mapping: the quad split at
    this size), 10 env-steps with given actions, bit-exact vs the oracle."""
    n, k = 4096, 10
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1)
    assert eng.cfg.LanesPerWalker == 0
    rng = np.random.default_rng(42)
    acts = rng.uniform(-1.1, 1.1, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e))) for e in range(n)]
    for i, e in enumerate(envs):
        for t in range(k):
            e.step(acts[t, i])
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    assert not fault.any()


def test_baseline_config3_rollout_update_4096(wk, orc):
    """BASELINE config 3: 4,096 walkers, full rollout + PPO update on one GPU: the
    recorded actions replay bit-exactly through the oracle's physics, and the update
    leaves finite weights that moved."""
    n, T = 4096, 8
    eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, Minibatch=4096, Epochs=2)
    w0 = eng.get_weights()
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e))) for e in range(n)]
    for i, e in enumerate(envs):
        for t in range(T):
            o, r, d = e.step(tr["actions"][t, i])
            assert r == tr["rewards"][t, i] and d == tr["dones"][t, i]
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    eng.ppo_update(update_index=0)
    w1 = eng.get_weights()
    assert np.isfinite(w1).all() and not np.array_equal(w0, w1)


def test_collective_path_matches_single_gpu_path(wk):
    """The multi-GPU minibatch sequence (ordered reduction -> RCCL all-reduce -> Adam) run
    through a one-rank communicator gives the same weights, Adam moments and diagnostics,
    bit for bit, as the single-GPU fused reduction+Adam: the RCCL path of bench.py --gpus N
    exercised on one device"""
    n, T = 4096, 16
    mk = lambda: wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, Minibatch=n // 4, Epochs=2)
    a, b = mk(), mk()
    b.comm_init(0, 1, wk.Engine.comm_unique_id())
    out = []
    for eng in (a, b):
        eng.rollout(T)
        d = eng.ppo_update(update_index=0)
        eng.rollout(T)
        d2 = eng.ppo_update(update_index=1)
        out.append((eng.get_weights(), eng.get_adam(), d, d2))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for x, y in zip(out[0][1], out[1][1]):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    assert out[0][2] == out[1][2] and out[0][3] == out[1][3]
    np.testing.assert_array_equal(a.get_state(), b.get_state())


@pytest.mark.parametrize("n", [1500, 5000, 8193])
def test_quad_walkers_per_wave_ragged(wk, orc, n):
    """the quad mapping's walkers per wave follow n (2 at 1,500, 8 at 5,000, 16 at 8,193; the
    last wave partial in each): physics bit-exact against the oracle"""
    k = 12
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, LanesPerWalker=4)
    envs, _, _ = oracle_envs(orc, eng, n)
    acts = np.random.default_rng(n).uniform(-1.2, 1.2, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
            np.testing.assert_array_equal(o, obs[t, i])
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    assert not fault.any()


def test_quad_sparse_equals_dense(wk, monkeypatch):
    """at the 8-GPU shard (8,192 walkers) the sparse quad mapping (eight walkers per wave, the
    other lanes replaying them) and the dense one (sixteen per wave, WK_QUAD_SPARSE=0) give the
    same policy rollout bit for bit: trajectory, returns and final state"""
    n, T = 8192, 24
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Horizon=T)
    monkeypatch.setenv("WK_QUAD_SPARSE", "0")
    dense = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Horizon=T)
    for x in (eng, dense):
        x.rollout(T)
    a, b = eng.get_trajectory(T), dense.get_trajectory(T)
    for key in a:
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
    np.testing.assert_array_equal(eng.get_state(), dense.get_state())
