// NativeMethods.cs -- P/Invoke binding of libwk.so (include/wk_api.h) for the reference's C#
// host (De-Rosa/PPO-BipedalWalker, .NET >= 6).  Every entry point of the C ABI is declared
// here with the header's parameter order; every struct mirrors the header's sequential layout
// (tests/test_csharp_binding.py checks both against include/wk_api.h and the ctypes layouts,
// since no .NET SDK exists in the build container).
//
// Conventions (wk_api.h): every call returns 0 or a negative wk_status; the message is
// wk_last_error(ctx) (ctx = IntPtr.Zero for wk_create failures) and the host logs it and
// continues, as every try/catch -> ErrorLogger.LogError does in the reference.  Arrays are
// caller-owned and copied during the call; a null array is passed as null.
using System;
using System.Runtime.InteropServices;

namespace NEA.Native;

public enum WkStatus { Ok = 0, Arg = -1, Hip = -2, Config = -3, Comm = -4, State = -5 }

public enum WkMaterial { Carpet = 0, Ice = 1, Rubber = 2, Metal = 3, Wood = 4, Paper = 5, Titanium = 6, SuperRubber = 7 }

public enum WkShape { Square = 0, Triangle = 1, Hexagon = 2 }

public static class WkConst
{
    public const int StateFloats = 112, NParam = 6149, NParamCritic = 897, NParamActor = 5252;
    public const int Obs = 12, Act = 4, NPairs = 9, MaxProps = 4, PropMaxV = 24, NEvents = 16;
    public const int IpcHandleBytes = 128;  // WK_IPC_HANDLE_BYTES: IPC handle + the GPU's PCI bus id
}

// Hyperparameters.cs:80-121 names and defaults (wk_config_defaults) + the batched extensions
[StructLayout(LayoutKind.Sequential)]
public struct WkConfig
{
    public int GameSpeed, Iterations, MaxTimesteps, RoughFloor, Epochs, BatchSize, UseGAE,
               NormalizeAdvantages;
    public float Gamma, Lambda, Epsilon, LogStandardDeviation, Alpha, Beta1, Beta2, AdamEpsilon;
    public IntPtr CriticNeuralNetwork, ActorNeuralNetwork;  // NULL = the default networks
    public float DeltaTime;
    public int Horizon, Minibatch, MinibatchGlobal, EnvOffset, RandomizeStart, RandomizeMaterial;
    public int LanesPerWalker;  // 0 = auto (4-lane split leg pairs up to 16,384 walkers, else the 2-lane leg split; 16-lane rows with RoughFloor)
}

// SerializableHyperparameters' host-only fields (Hyperparameters.cs:11-77)
[StructLayout(LayoutKind.Sequential, CharSet = CharSet.Ansi)]
public struct WkHostSettings
{
    public int CollectData, SaveWeights;
    [MarshalAs(UnmanagedType.ByValTStr, SizeConst = 256)] public string CriticNeuralNetwork;
    [MarshalAs(UnmanagedType.ByValTStr, SizeConst = 256)] public string ActorNeuralNetwork;
    [MarshalAs(UnmanagedType.ByValTStr, SizeConst = 256)] public string CriticWeightFileName;
    [MarshalAs(UnmanagedType.ByValTStr, SizeConst = 256)] public string ActorWeightFileName;
    [MarshalAs(UnmanagedType.ByValTStr, SizeConst = 1024)] public string FilePath;
}

// per-substep pair bookkeeping (wk_step_traced)
[StructLayout(LayoutKind.Sequential)]
public unsafe struct WkPairTrace
{
    public fixed byte AabbHit[9];
    public fixed byte SatHit[9];
    public fixed byte NContacts[9];
    public fixed byte Pad[5];
    public fixed float Normal[18];
    public fixed float Depth[9];
    public fixed float Contact[36];
    public fixed float Impulse[18];
    public fixed float JointDepth[4];
    public fixed float JointImpulse[4];
}

// one body of one walker, for Renderer.RenderRigidObject / ConsoleRenderer
[StructLayout(LayoutKind.Sequential)]
public unsafe struct WkBodyView
{
    public int NVertices;
    public fixed float Vertices[12];
    public fixed float Centroid[2];
    public fixed float LinearVelocity[2];
    public float AngularVelocity, Angle;
    public int Collided, IsStatic;
}

// Square / Triangle / Hexagon.FromSize(...).SmoothCorners(...) + velocities, acceleration
[StructLayout(LayoutKind.Sequential)]
public struct WkProp
{
    public int Shape, Smooth, Material, IsStatic;
    public float Cx, Cy, Size;
    public float Vx, Vy, W;
    public float Ax, Ay;
}

[StructLayout(LayoutKind.Sequential)]
public unsafe struct WkPropView
{
    public int NVertices;
    public fixed float Vertices[48];
    public fixed float Centroid[2];
    public fixed float LinearVelocity[2];
    public float AngularVelocity, Angle;
    public int IsStatic;
}

[StructLayout(LayoutKind.Sequential)]
public struct WkPpoArgs
{
    public int Epochs, Minibatch, MinibatchGlobal;
    public uint UpdateIndex;
}

[StructLayout(LayoutKind.Sequential)]
public struct WkRolloutStats
{
    public double RewardSum;
    public long Episodes, EnvSteps;
    public uint FaultOr;
    public int Pad;
}

[StructLayout(LayoutKind.Sequential)]
public struct WkEpisodeRec
{
    public float TotalReward;
    public int Env, Length;
    public uint Step;
}

[StructLayout(LayoutKind.Sequential)]
public struct WkProfile
{
    public double PhysicsMs; public long PhysicsLaunches; public long PhysicsEnvSteps;
    public double GradMs; public long GradLaunches;
    public double ReduceMs; public long ReduceLaunches;
    public double AdamMs; public long AdamLaunches;
    public double AllreduceMs; public long AllreduceCalls;
    public double ReturnsMs; public long ReturnsLaunches;
    public double UpdateMs; public long UpdateCalls;
}

public static class Wk
{
    const string Lib = "wk";  // libwk.so next to the executable (or on LD_LIBRARY_PATH)

    [DllImport(Lib)] public static extern void wk_config_defaults(ref WkConfig cfg);
    [DllImport(Lib)] public static extern IntPtr wk_version();
    [DllImport(Lib)] public static extern int wk_create(ref WkConfig cfg, int device, int nEnv, ulong seed, out IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_destroy(IntPtr ctx);
    [DllImport(Lib)] public static extern IntPtr wk_last_error(IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_sync(IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_num_envs(IntPtr ctx);

    // environment
    [DllImport(Lib)] public static extern int wk_reset(IntPtr ctx, byte[]? mask);
    [DllImport(Lib)] public static extern int wk_set_materials(IntPtr ctx, int[] matId);
    [DllImport(Lib)] public static extern int wk_set_offsets(IntPtr ctx, float[] dx);
    [DllImport(Lib)] public static extern int wk_step(IntPtr ctx, float[]? actions, int kSteps, float[]? obs, float[]? reward, byte[]? done, uint[]? fault);
    [DllImport(Lib)] public static extern int wk_step_sampled(IntPtr ctx, int kSteps, float[]? states, float[]? actions, float[]? logp, float[]? values, float[]? reward, byte[]? done, float[]? nextObs, uint[]? fault, float[]? position);
    [DllImport(Lib)] public static extern int wk_step_device(IntPtr ctx, IntPtr dActions, int kSteps, IntPtr dObs, IntPtr dReward, IntPtr dDone, IntPtr dFault);
    [DllImport(Lib)] public static extern int wk_step_traced(IntPtr ctx, float[] actions, [Out] WkPairTrace[] trace);
    [DllImport(Lib)] public static extern int wk_get_obs(IntPtr ctx, float[] obs);
    [DllImport(Lib)] public static extern int wk_get_state(IntPtr ctx, float[] state);
    [DllImport(Lib)] public static extern int wk_set_state(IntPtr ctx, float[] state);
    [DllImport(Lib)] public static extern int wk_check_state(float[] state, int nEnv, out int badEnv, out int badBody);
    [DllImport(Lib)] public static extern int wk_take_actions(IntPtr ctx, int env, float[] actions);
    [DllImport(Lib)] public static extern int wk_object_update(IntPtr ctx, int listCount, float deltaTime);
    [DllImport(Lib)] public static extern int wk_joint_step(IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_body_order(IntPtr ctx, int env, int[] parts, out int count);
    [DllImport(Lib)] public static extern int wk_get_body_view(IntPtr ctx, int env, int body, out WkBodyView view);
    [DllImport(Lib)] public static extern int wk_set_scene(IntPtr ctx, WkProp[]? props, int nProps);
    [DllImport(Lib)] public static extern int wk_get_prop_view(IntPtr ctx, int env, int prop, out WkPropView view);

    // weights, configuration, checkpoints
    [DllImport(Lib)] public static extern int wk_get_weights(IntPtr ctx, float[] p);
    [DllImport(Lib)] public static extern int wk_set_weights(IntPtr ctx, float[] p);
    [DllImport(Lib)] public static extern int wk_get_adam(IntPtr ctx, float[]? m, float[]? v, out int t);
    [DllImport(Lib)] public static extern int wk_set_adam(IntPtr ctx, float[]? m, float[]? v, int t);
    [DllImport(Lib)] public static extern void wk_host_settings_defaults(ref WkHostSettings host);
    [DllImport(Lib)] public static extern int wk_config_to_json(ref WkConfig cfg, ref WkHostSettings host, byte[] text, UIntPtr cap);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_config_from_json(string json, ref WkConfig cfg, ref WkHostSettings host);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_config_save_json(string path, ref WkConfig cfg, ref WkHostSettings host);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_config_load_json(string path, ref WkConfig cfg, ref WkHostSettings host);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_save_weights(IntPtr ctx, string criticPath, string actorPath);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_load_weights(IntPtr ctx, string criticPath, string actorPath);
    [DllImport(Lib)] public static extern int wk_format_weights(float[] p, byte[] critic, UIntPtr criticCap, byte[] actor, UIntPtr actorCap);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_parse_weights(string critic, string actor, float[] p);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_checkpoint_save(IntPtr ctx, string path);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_checkpoint_load(IntPtr ctx, string path);

    // agent
    [DllImport(Lib)] public static extern int wk_policy_sample(IntPtr ctx, int n, float[] obs, int[]? envIds, uint[]? steps, float[]? mean, float[]? act, float[]? logp);
    [DllImport(Lib)] public static extern int wk_value(IntPtr ctx, int n, float[] obs, float[] v);

    // rollout + PPO
    [DllImport(Lib)] public static extern int wk_rollout(IntPtr ctx, int horizon);
    [DllImport(Lib)] public static extern int wk_rollout_stats_get(IntPtr ctx, out WkRolloutStats stats);
    [DllImport(Lib)] public static extern int wk_get_trajectory(IntPtr ctx, float[]? states, float[]? actions, float[]? logp, float[]? rewards, byte[]? dones, float[]? values, float[]? returns, float[]? advantages);
    [DllImport(Lib)] public static extern int wk_set_trajectory(IntPtr ctx, int horizon, float[] states, float[] actions, float[] logp, float[] rewards, byte[] dones, float[] values);
    [DllImport(Lib)] public static extern int wk_compute_returns(IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_ppo_update(IntPtr ctx, ref WkPpoArgs args, out float criticDiag, out float actorDiag);
    [DllImport(Lib)] public static extern int wk_train_batch(IntPtr ctx, int B, float bDiv, float[] states, float[] actions, float[] logpOld, float[] returns, float[] adv, out float criticDiag, out float actorDiag, float[]? gradsOut, int applyAdam, out int skipped);
    [DllImport(Lib)] public static extern int wk_minibatch_gradient(IntPtr ctx, int B, float bDiv, float[] states, float[] actions, float[] logpOld, float[] returns, float[] adv, out float criticDiag, out float actorDiag, float[]? gradsOut, out int skipped);

    // data collection (ConsoleRenderer.AddTotalEpisodeReward / AddCriticLoss / AddActorLoss / CreateDataFile)
    [DllImport(Lib)] public static extern int wk_collect_data(IntPtr ctx, int on);
    [DllImport(Lib)] public static extern int wk_episode_log_count(IntPtr ctx, out long episodes, out long updates);
    [DllImport(Lib)] public static extern int wk_episode_log_drain(IntPtr ctx, [Out] WkEpisodeRec[] recs, long cap, out long n, out long dropped);
    [DllImport(Lib)] public static extern int wk_loss_log_drain(IntPtr ctx, float[] critic, float[] actor, long cap, out long n, out long dropped);
    [DllImport(Lib, CharSet = CharSet.Ansi)] public static extern int wk_write_data_file(string path, float[] totalRewards, long nRewards, float[] criticLosses, long nCritic, float[] actorLosses, long nActor);

    // multi-GPU (one process per GPU)
    [DllImport(Lib)] public static extern int wk_comm_unique_id(byte[] id);
    [DllImport(Lib)] public static extern int wk_comm_init(IntPtr ctx, int rank, int nRanks, byte[] uniqueId);
    [DllImport(Lib)] public static extern int wk_allreduce_test(IntPtr ctx, float[] buf, int n);
    [DllImport(Lib)] public static extern int wk_comm_ipc_handle(IntPtr ctx, byte[] handle);
    [DllImport(Lib)] public static extern int wk_comm_init_ipc(IntPtr ctx, int rank, int nRanks, byte[] handles);
    [DllImport(Lib)] public static extern int wk_comm_info(IntPtr ctx, out int kind, out int flags);
    [DllImport(Lib)] public static extern int wk_comm_set_timeout(IntPtr ctx, double seconds);
    [DllImport(Lib)] public static extern int wk_comm_xch_profile(IntPtr ctx, int minibatches);
    [DllImport(Lib)] public static extern int wk_comm_xch_stamps(IntPtr ctx, ulong[] stamps, int maxLaunches, out int launches, out int blocks);
    [UnmanagedFunctionPointer(CallingConvention.Cdecl)] public delegate int HostAllReduce(IntPtr buf, int n, IntPtr user);
    [DllImport(Lib)] public static extern int wk_comm_init_host(IntPtr ctx, int rank, int nRanks, HostAllReduce fn, IntPtr user);

    // libwk keeps the function pointer for the context's lifetime; the marshalled thunk dies with
    // the delegate, so the delegate must stay reachable until the context is destroyed.  Use
    // CommInitHost / Destroy instead of the raw entry points when a host all-reduce is set.
    // A failing callback (non-zero return) fails that rank's wk_ppo_update with WK_ERR_COMM
    // while its peers wait in their own all-reduce: treat it as fatal for the whole job.
    static readonly System.Collections.Concurrent.ConcurrentDictionary<IntPtr, HostAllReduce> s_hostAllReduce = new();
    public static int CommInitHost(IntPtr ctx, int rank, int nRanks, HostAllReduce fn, IntPtr user)
    {
        int rc = wk_comm_init_host(ctx, rank, nRanks, fn, user);
        if (rc == 0) s_hostAllReduce[ctx] = fn;
        return rc;
    }
    public static int Destroy(IntPtr ctx)
    {
        int rc = wk_destroy(ctx);
        s_hostAllReduce.TryRemove(ctx, out _);
        return rc;
    }

    // profiling, counting replay, snapshots
    [DllImport(Lib)] public static extern int wk_profile_enable(IntPtr ctx, int on);
    [DllImport(Lib)] public static extern int wk_profile_get(IntPtr ctx, out WkProfile profile);
    [DllImport(Lib)] public static extern int wk_profile_reset(IntPtr ctx);
    [DllImport(Lib)] public static extern int wk_count_events(IntPtr ctx, int k, ulong[] counts);
    [DllImport(Lib)] public static extern int wk_snapshot(IntPtr ctx, int op);
    [DllImport(Lib)] public static extern int wk_time_gradient(IntPtr ctx, int minibatch, int reps, out double msPerLaunch);
    [DllImport(Lib)] public static extern int wk_time_gradient_ex(IntPtr ctx, int minibatch, int reps, int flags, out double msPerLaunch);
    [DllImport(Lib)] public static extern int wk_rollout_mapping(IntPtr ctx, out int lanesPerWalker, out int walkersPerWave, out long waves, out long wavesLaunched);
    [DllImport(Lib)] public static extern int wk_grad_kernel(IntPtr ctx, int minibatch);

    public static string LastError(IntPtr ctx) => Marshal.PtrToStringAnsi(wk_last_error(ctx)) ?? "";

    // log-and-continue, like every try/catch -> ErrorLogger.LogError in the reference
    public static bool Ok(IntPtr ctx, int rc, string what, Action<string>? log = null)
    {
        if (rc == 0) return true;
        (log ?? Console.Error.WriteLine)($"{what}: {LastError(ctx)} ({(WkStatus)rc})");
        return false;
    }
}
