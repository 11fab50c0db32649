// Api.cs -- the reference's object API (IMaterial, IObject, RigidBody, Walker) over libwk.so, so a
// C# host that used NEA.Materials / NEA.Objects / NEA.Walker keeps compiling against the same
// names: Materials/IMaterial.cs:6-12 and the eight materials, Objects/IObject.cs:7-10,
// Bodies/RigidBody.cs (the read side a renderer and GetState use), Walker/Walker.cs:49-223.
// The C++ mirror of the same surface is csrc/host/nea.hpp; this file follows it member for
// member.  The physics state lives on the GPU (one context per environment), so a RigidBody
// here is a view of one body of one walker (wk_get_body_view).  A host that keeps the reference's
// Environment.StepObjects loop (Environment.cs:126-143: per substep Joint.Step on the 4 joints,
// then IObject.Update on every body of the list) calls wk_object_update list.Count * Iterations
// times per frame: the frame's first call runs the env-step of every walker with the torques
// Walker.TakeActions stored (wk_take_actions), the others are counted no-ops.  Errors are logged
// and the operation skipped (ErrorLogger.LogError, the reference's convention).
using System;
using System.Collections.Generic;

namespace NEA.Materials
{
    // Materials/IMaterial.cs:6-12 (Color omitted: headless); Id selects the kernel's table
    public interface IMaterial
    {
        float InverseMass { get; }
        float Friction { get; }
        float Restitution { get; }
        int Id { get; }
    }
    // Materials/<Name>.cs: the constants of csrc/wk_common.h material() and nea.hpp
    public sealed class Carpet : IMaterial { public float InverseMass => 5f; public float Friction => 0.8f; public float Restitution => 0.3f; public int Id => 0; }
    public sealed class Ice : IMaterial { public float InverseMass => 11f; public float Friction => 0f; public float Restitution => 0.3f; public int Id => 1; }
    public sealed class Rubber : IMaterial { public float InverseMass => 11f; public float Friction => 0.5f; public float Restitution => 0.7f; public int Id => 2; }
    public sealed class Metal : IMaterial { public float InverseMass => 15f; public float Friction => 1f; public float Restitution => 0.3f; public int Id => 3; }
    public sealed class Wood : IMaterial { public float InverseMass => 20f; public float Friction => 0.01f; public float Restitution => 0.3f; public int Id => 4; }
    public sealed class Paper : IMaterial { public float InverseMass => 1f; public float Friction => 0.1f; public float Restitution => 0.3f; public int Id => 5; }
    public sealed class Titanium : IMaterial { public float InverseMass => 0.01f; public float Friction => 0.2f; public float Restitution => 0.1f; public int Id => 6; }
    public sealed class SuperRubber : IMaterial { public float InverseMass => 11f; public float Friction => 1f; public float Restitution => 1f; public int Id => 7; }
}

namespace NEA.Objects
{
    using NEA.Bodies;

    // Objects/IObject.cs:7-10
    public interface IObject
    {
        void Update(List<RigidBody> rigidBodies, float deltaTime);
    }
}

namespace NEA.Bodies
{
    using NEA.Native;
    using NEA.Objects;

    // Bodies/RigidBody.cs, the read side (GetVertices / GetCentroid / GetLinearVelocity /
    // GetAngularVelocity / GetAngle / Collided / IsStatic) of body `Part` (0 LLL, 1 LLU, 2 Body,
    // 3 RLL, 4 RLU, 5 Floor -- 5..14 the rough floor's segments) of walker `Env`.
    // Update (IObject): the GPU resolves every body of the list in the reference's order inside
    // one env-step, so stepping one body alone does not exist; the frame is assembled natively.
    public sealed class RigidBody : IObject
    {
        readonly IntPtr _ctx;
        public int Env { get; }
        public int Part { get; }
        internal RigidBody(IntPtr ctx, int env, int part) { _ctx = ctx; Env = env; Part = part; }

        WkBodyView View()
        {
            Wk.Ok(_ctx, Wk.wk_get_body_view(_ctx, Env, Part, out var v), "Exception while reading a rigid body", Console.Error.WriteLine);
            return v;
        }
        public unsafe List<(float X, float Y)> GetVertices()
        {
            var v = View();
            var l = new List<(float, float)>(v.NVertices);
            for (int i = 0; i < v.NVertices; i++) l.Add((v.Vertices[2 * i], v.Vertices[2 * i + 1]));
            return l;
        }
        public unsafe (float X, float Y) GetCentroid() { var v = View(); return (v.Centroid[0], v.Centroid[1]); }
        public unsafe (float X, float Y) GetLinearVelocity() { var v = View(); return (v.LinearVelocity[0], v.LinearVelocity[1]); }
        public float GetAngularVelocity() => View().AngularVelocity;
        public float GetAngle() => View().Angle;
        public bool Collided => View().Collided != 0;
        public bool IsStatic => View().IsStatic != 0;

        // IObject.Update (Objects/IObject.cs:9), called list.Count * Iterations times per frame by
        // Environment.StepObjects (Environment.cs:130-141): the frame's first call steps every
        // walker of the context once with the torques Walker.TakeActions stored (a walker given
        // none keeps its torques: no kick), the frame's other calls are no-ops (wk_object_update)
        public void Update(List<RigidBody> rigidBodies, float deltaTime)
        {
            int r = Wk.wk_object_update(_ctx, rigidBodies.Count, deltaTime);
            if (r < 0) Wk.Ok(_ctx, r, "Exception occurred during the environment update", Console.Error.WriteLine);
        }
    }

    // Joint.Step (Joint.cs:31-41): the joints of every walker are resolved inside the frame's
    // env-step (wk_joint_step is a no-op kept for the call shape)
    public sealed class Joint
    {
        readonly IntPtr _ctx;
        internal Joint(IntPtr ctx) { _ctx = ctx; }
        public void Step() => Wk.wk_joint_step(_ctx);
    }
}

namespace NEA.Walker
{
    using NEA.Bodies;
    using NEA.Materials;
    using NEA.Native;
    using NEA.Objects;

    // Walker/Walker.cs:49-223 for walker `Index` of a context (a Walker owns no state of its own:
    // its bodies, torques, Collided flags and episode counter live in the context's records)
    public sealed class Walker
    {
        readonly IntPtr _ctx;
        readonly Action<string> _log;
        public int Index { get; }
        public IMaterial Material { get; }

        public Walker(IntPtr ctx, int index, IMaterial? material = null, Action<string>? log = null)
        {
            _ctx = ctx;
            Index = index;
            _log = log ?? Console.Error.WriteLine;
            Material = material ?? new Carpet();  // Walker.cs:28 (_material = new Carpet())
        }

        // CreateCreature (Walker.cs:38-44): the context created every walker's bodies, joints,
        // associated bodies and gravity at wk_create (the materials: wk_set_materials, from the
        // host's IMaterial.Id per walker); this fills the caller's list with the walker's bodies
        public void CreateCreature(List<RigidBody> rigidBodies)
        {
            rigidBodies.Clear();
            rigidBodies.AddRange(Bodies());
        }

        // the list RigidBody.ResolveCollisions walks, in its current order (wk_body_order):
        // [LLL, LLU, Body, RLL, RLU, Floor] in episode 0, [Floor, LLL, LLU, Body, RLL, RLU] after a
        // reset (Reset removes the walker's bodies and CreateBodies appends them after the floor,
        // Walker.cs:191-234); the rough floor's ten segments stand where the floor does
        public List<RigidBody> Bodies()
        {
            var parts = new int[15];
            var l = new List<RigidBody>(15);
            if (!Wk.Ok(_ctx, Wk.wk_body_order(_ctx, Index, parts, out int n), "Exception while reading the body list", _log))
                return l;
            for (int i = 0; i < n; i++) l.Add(new RigidBody(_ctx, Index, parts[i]));
            return l;
        }

        // the part of this walker's list (by part id, whatever the list order)
        RigidBody Part(int part) => new RigidBody(_ctx, Index, part);

        // GetJoints (Walker.cs:102): [bodyJointLeft, bodyJointRight, leftJoint, rightJoint]
        public List<Joint> GetJoints() => new List<Joint> { new(_ctx), new(_ctx), new(_ctx), new(_ctx) };

        // Walker.Update (:49-54): terminal once the body or an upper leg touched the floor
        public bool Terminal => Part(2).Collided || Part(1).Collided || Part(4).Collided;

        // GetActions (:57-62): the policy's sample for this walker's state
        public float[] GetActions(float[] state, out float[] logProbabilities)
        {
            var a = new float[WkConst.Act];
            var mean = new float[WkConst.Act];
            logProbabilities = new float[WkConst.Act];
            var ids = new[] { Index };
            Wk.Ok(_ctx, Wk.wk_policy_sample(_ctx, 1, state, ids, null, mean, a, logProbabilities),
                  "Exception thrown while attempting to sample actions", _log);
            return a;
        }

        // TakeActions (:66-75): the torques of the next frame; a wrong-sized action is ignored
        // like the reference's height check; the joints' SetTorque runs inside the step
        public void TakeActions(float[] actions)
        {
            if (actions.Length != WkConst.Act) return;
            Wk.Ok(_ctx, Wk.wk_take_actions(_ctx, Index, actions), "Exception while setting the torques", _log);
        }

        // GetState (:132-152)
        public float[] GetState()
        {
            int n = Wk.wk_num_envs(_ctx);
            var all = new float[n * WkConst.Obs];
            var s = new float[WkConst.Obs];
            if (Wk.Ok(_ctx, Wk.wk_get_obs(_ctx, all), "Exception while reading the walker state", _log))
                Array.Copy(all, Index * WkConst.Obs, s, 0, WkConst.Obs);
            return s;
        }

        // GetPosition (:108-111): the torso's centroid
        public (float X, float Y) GetPosition() => Part(2).GetCentroid();

        // Reset (:212-223): this walker back to its template (post-reset list order)
        public void Reset(List<RigidBody> rigidBodies)
        {
            var mask = new byte[Wk.wk_num_envs(_ctx)];
            mask[Index] = 1;
            Wk.Ok(_ctx, Wk.wk_reset(_ctx, mask), "Exception while resetting the walker", _log);
            rigidBodies.Clear();
            rigidBodies.AddRange(Bodies());
        }
    }
}
