// HeadlessEnvironment.cs -- the reference's Environment (Environment.cs:18-226) for one walker,
// headless (no SpriteBatch / Renderer, no Console.KeyAvailable), on libwk.so.  The public
// surface follows the reference: Update(deltaTime), InitialState(), GetConsoleInformation(),
// and the trajectory it records per frame is exactly Environment.cs:70-89's -- the state
// observed before the step, the UNCLIPPED sampled action and its per-dimension
// log-probabilities (wk_step_sampled), the reward -- so TrainNetworks (:157-164) trains on the
// same Trajectory through PPOAgent.Train's batched equivalent (wk_set_trajectory +
// wk_ppo_update: returns / advantages, Epochs x floor(T / BatchSize) minibatches, Adam).
using System;
using System.Collections.Generic;
using System.Linq;

namespace NEA.Native;

// Walker/PPO/Trajectory.cs:7-30, flat float rows instead of List<Matrix>
public sealed class Trajectory
{
    public readonly List<float[]> States = new(), Actions = new(), LogProbabilities = new();
    public readonly List<float> Rewards = new(), Values = new();
    public readonly List<int> Indexes = new();
}

public sealed class HeadlessEnvironment : IDisposable
{
    readonly IntPtr _ctx;
    readonly WkConfig _cfg;
    readonly Action<string> _log;
    Trajectory _trajectory = new();
    float[] _state = new float[WkConst.Obs];

    // Environment.cs:31-35
    int _steps = 0;
    int _episodes = 0;
    float _bestDistance = 0;
    float _previousAverageReward = 0;

    // Hyperparameters.CollectData: ConsoleRenderer.AddTotalEpisodeReward / AddCriticLoss /
    // AddActorLoss only append when it is set (ConsoleRenderer.cs:79-95)
    public bool CollectData { get; set; } = true;
    public List<float> TotalRewards { get; } = new();  // ConsoleRenderer._totalRewards
    public List<float> CriticLosses { get; } = new();  // ConsoleRenderer._criticLosses
    public List<float> ActorLosses { get; } = new();   // ConsoleRenderer._actorLosses

    // Environment(SpriteBatch, Renderer) (:39-51): Walker + CreateCreature + CreateFloor + agent
    public HeadlessEnvironment(ulong seed = 20250905, int device = 0, Action<string>? log = null,
                               Func<WkConfig, WkConfig>? configure = null)
    {
        _log = log ?? Console.Error.WriteLine;
        var c = new WkConfig();
        Wk.wk_config_defaults(ref c);          // Hyperparameters.cs:83-121 defaults
        if (configure != null) c = configure(c);
        c.Horizon = c.MaxTimesteps + 1;        // one whole episode (terminal at steps > MaxTimesteps)
        c.Minibatch = c.BatchSize;             // CreateBatches draws BatchSize samples
        c.MinibatchGlobal = c.BatchSize;
        _cfg = c;
        if (Wk.wk_create(ref c, device, 1, seed, out _ctx) != 0)
            throw new InvalidOperationException($"wk_create: {Wk.LastError(IntPtr.Zero)}");
        InitialState();
    }

    public void Dispose() => Wk.Destroy(_ctx);

    // InitialState (:175-180): Walker.Update + GetState
    public void InitialState()
    {
        Wk.Ok(_ctx, Wk.wk_get_obs(_ctx, _state), "Exception while reading the walker state", _log);
    }

    // Update (:64-92): observe -> sample -> clip + TakeActions -> Step -> record; train at the end
    public void Update(float deltaTime)
    {
        _trajectory.Indexes.Add(_steps);
        _steps++;
        var s = new float[WkConst.Obs];
        var a = new float[WkConst.Act];
        var lp = new float[WkConst.Act];
        var v = new float[1];
        var r = new float[1];
        var d = new byte[1];
        var next = new float[WkConst.Obs];
        var pos = new float[2];
        // deltaTime: the context steps with its configured DeltaTime (Game1's fixed step)
        if (!Wk.Ok(_ctx, Wk.wk_step_sampled(_ctx, 1, s, a, lp, v, r, d, next, null, pos),
                   "Exception occurred during the environment update", _log))
            return;
        _trajectory.States.Add(s);             // == _state (:73)
        _trajectory.Actions.Add(a);            // the unclipped action (:86)
        _trajectory.LogProbabilities.Add(lp);  // (:87)
        _trajectory.Rewards.Add(r[0]);         // (:88)
        _trajectory.Values.Add(v[0]);
        _state = next;
        // Step (:119) reads the position after the step and before Reset: the context has
        // already re-created a terminal walker, so the pre-reset position comes from the step
        if (pos[0] > _bestDistance) _bestDistance = pos[0];
        if (d[0] != 0) TrainNetworks();
    }

    // TrainNetworks (:157-164) -> Walker.Train -> PPOAgent.Train(Trajectory) (PPOAgent.cs:147-172)
    void TrainNetworks()
    {
        _episodes++;
        _previousAverageReward = _trajectory.Rewards.Average();
        int T = _trajectory.Rewards.Count;
        if (CollectData) TotalRewards.Add((float)_trajectory.Rewards.Sum(x => (double)x));  // PPOAgent.cs:151
        var S = _trajectory.States.SelectMany(x => x).ToArray();
        var A = _trajectory.Actions.SelectMany(x => x).ToArray();
        var L = _trajectory.LogProbabilities.SelectMany(x => x).ToArray();
        var R = _trajectory.Rewards.ToArray();
        var V = _trajectory.Values.ToArray();
        var D = new byte[T];
        D[T - 1] = 1;                          // one episode: returns restart after it
        // PPOAgent.cs:153-166: valueLoss / actorLoss start at 0 and keep the last minibatch's
        // diagnostics; with floor(T / BatchSize) == 0 minibatches no Train(Batch) runs and the
        // zeros are appended all the same
        float critic = 0, actor = 0;
        if (Wk.Ok(_ctx, Wk.wk_set_trajectory(_ctx, T, S, A, L, R, D, V), "Exception while storing the trajectory", _log)
            && T >= _cfg.BatchSize)
        {
            var args = new WkPpoArgs { Epochs = _cfg.Epochs, Minibatch = _cfg.BatchSize,
                                       MinibatchGlobal = _cfg.BatchSize, UpdateIndex = (uint)(_episodes - 1) };
            if (!Wk.Ok(_ctx, Wk.wk_ppo_update(_ctx, ref args, out critic, out actor),
                       "Exception while training the networks", _log))
                critic = actor = 0;
        }
        if (CollectData)
        {
            CriticLosses.Add(critic);          // ConsoleRenderer.AddCriticLoss (PPOAgent.cs:165)
            ActorLosses.Add(actor);            // ConsoleRenderer.AddActorLoss (:166)
        }
        Reset();
    }

    // Reset (:167-173): the context has re-created the walker in the post-reset body order
    void Reset()
    {
        _trajectory = new Trajectory();
        _steps = 0;
    }

    // GetConsoleInformation (:56-60)
    public (int, int, float, float, float, float, float[]) GetConsoleInformation()
    {
        float averageReward = _trajectory.Rewards.Count == 0 ? 0 : _trajectory.Rewards.Average();
        return (_episodes, _steps, GetPosition().x, averageReward, _bestDistance, _previousAverageReward, _state);
    }

    // Walker.GetPosition (Walker.cs:49-54): the torso's centroid
    public (float x, float y) GetPosition()
    {
        if (!Wk.Ok(_ctx, Wk.wk_get_body_view(_ctx, 0, 2, out var body), "Exception while reading the walker", _log))
            return (0, 0);
        unsafe { return (body.Centroid[0], body.Centroid[1]); }
    }

    // the six bodies Renderer.RenderRigidObject draws (LLL, LLU, Body, RLL, RLU, Floor)
    public WkBodyView[] Bodies()
    {
        var views = new WkBodyView[6];
        for (int b = 0; b < 6; b++) Wk.Ok(_ctx, Wk.wk_get_body_view(_ctx, 0, b, out views[b]), "Exception while reading a body", _log);
        return views;
    }

    // ConsoleRenderer.CreateDataFile (:124-135)
    public void CreateDataFile(string path) =>
        Wk.Ok(_ctx, Wk.wk_write_data_file(path, TotalRewards.ToArray(), TotalRewards.Count, CriticLosses.ToArray(),
                                          CriticLosses.Count, ActorLosses.ToArray(), ActorLosses.Count),
              "Exception while writing the data file", _log);

    // PPOAgent.Save / Load (PPOAgent.cs:192-213): the reference's text weights files
    public void Save(string criticPath, string actorPath) =>
        Wk.Ok(_ctx, Wk.wk_save_weights(_ctx, criticPath, actorPath), "Exception while attempting to save the critic and actor neural networks", _log);
    public void Load(string criticPath, string actorPath) =>
        Wk.Ok(_ctx, Wk.wk_load_weights(_ctx, criticPath, actorPath), "Exception while attempting to load the critic and actor neural networks", _log);
}
