// nea.hpp -- C++ host mirror of the reference's hot-path interface over the C ABI.
//
// Same names, argument meaning and error behaviour as the reference's managed API
// (namespace NEA in /root/reference), batched over N walker instances that live on one
// GPU.  Errors follow the reference's log-and-continue convention
// (Rendering/ErrorLogger.cs:42-78): a failing call is logged through the ErrorLogger
// hook and the operation is skipped; construction failures throw (the reference's ctor
// paths throw too).
//
//   NEA::Materials::IMaterial + Carpet/Ice/Rubber/...   Materials/<Name>.cs
//   NEA::Environment                                    Environment.cs:18-261
//     Update(deltaTime)      -> Environment.Update (:64-92) for all walkers
//     StepObjects(actions)   -> Environment.StepObjects (:126-143) under caller actions
//     InitialState()         -> Environment.InitialState (:176-180)
//     GetConsoleInformation  -> Environment.GetConsoleInformation (:56-60)
//   NEA::Walker::Walker                                 Walker/Walker.cs
//     GetState / TakeActions / GetPosition / body views
//   NEA::Walker::PPO::PPOAgent                          Walker/PPO/PPOAgent.cs
//     SampleActions (:381-398), Train (:147-172), GetValueEstimate (:350-364)
//   NEA::Walker::PPO::Hyperparameters                   Walker/PPO/Hyperparameters.cs:80-121
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include <sys/stat.h>

#include "../../../include/wk_api.h"

namespace NEA {

// ErrorLogger.LogError (Rendering/ErrorLogger.cs:42-45): replaceable sink
inline std::function<void(const std::string&)>& ErrorLoggerSink() {
  static std::function<void(const std::string&)> sink = [](const std::string& m) {
    std::fprintf(stderr, "[ErrorLogger] %s\n", m.c_str());
  };
  return sink;
}
inline void LogError(const std::string& m) { ErrorLoggerSink()(m); }

namespace Materials {
// IMaterial (Materials/IMaterial.cs:6-12); Id() selects the kernel's constant table
struct IMaterial {
  virtual ~IMaterial() = default;
  virtual float InverseMass() const = 0;
  virtual float Friction() const = 0;
  virtual float Restitution() const = 0;
  virtual int Id() const = 0;
};
#define NEA_MATERIAL(Name, id, im, fr, re)                      \
  struct Name : IMaterial {                                     \
    float InverseMass() const override { return im; }           \
    float Friction() const override { return fr; }              \
    float Restitution() const override { return re; }           \
    int Id() const override { return id; }                      \
  };
NEA_MATERIAL(Carpet, WK_MAT_CARPET, 5.0f, 0.8f, 0.3f)
NEA_MATERIAL(Ice, WK_MAT_ICE, 11.0f, 0.0f, 0.3f)
NEA_MATERIAL(Rubber, WK_MAT_RUBBER, 11.0f, 0.5f, 0.7f)
NEA_MATERIAL(Metal, WK_MAT_METAL, 15.0f, 1.0f, 0.3f)
NEA_MATERIAL(Wood, WK_MAT_WOOD, 20.0f, 0.01f, 0.3f)
NEA_MATERIAL(Paper, WK_MAT_PAPER, 1.0f, 0.1f, 0.3f)
NEA_MATERIAL(Titanium, WK_MAT_TITANIUM, 0.01f, 0.2f, 0.1f)
NEA_MATERIAL(SuperRubber, WK_MAT_SUPERRUBBER, 11.0f, 1.0f, 1.0f)
#undef NEA_MATERIAL
}  // namespace Materials

namespace Objects {
namespace RigidBodies {
// Square / Triangle / Hexagon (Objects/RigidBodies/<Shape>.cs): FromSize builds the
// description of one scene prop; the RigidBody setters the reference offers before the body
// joins the list (RigidBody.cs:143-189) fill in the rest.  Environment::AddRigidBodies
// hands them to every walker (wk_set_scene).
class Prop {
 public:
  Prop& SmoothCorners(int count = 1) { p_.smooth += count; return *this; }
  Prop& SetLinearVelocity(float x, float y) { p_.vx = x; p_.vy = y; return *this; }
  Prop& SetAngularVelocity(float w) { p_.w = w; return *this; }
  Prop& AddAcceleration(float x, float y) { p_.ax = p_.ax + x; p_.ay = p_.ay + y; return *this; }
  const wk_prop& Desc() const { return p_; }

 protected:
  Prop(int shape, const Materials::IMaterial& m, float cx, float cy, float size, bool isStatic) {
    p_.shape = shape; p_.smooth = 0; p_.material = m.Id(); p_.is_static = isStatic ? 1 : 0;
    p_.cx = cx; p_.cy = cy; p_.size = size;
    p_.vx = p_.vy = p_.w = p_.ax = p_.ay = 0.0f;
  }
  wk_prop p_{};
};
#define NEA_SHAPE(Name, id)                                                                   \
  struct Name : Prop {                                                                        \
    static Name FromSize(const Materials::IMaterial& m, float cx, float cy, float size,       \
                         bool isStatic = false) {                                             \
      return Name(m, cx, cy, size, isStatic);                                                 \
    }                                                                                         \
                                                                                              \
   private:                                                                                   \
    Name(const Materials::IMaterial& m, float cx, float cy, float size, bool st)              \
        : Prop(id, m, cx, cy, size, st) {}                                                    \
  };
NEA_SHAPE(Square, WK_SHAPE_SQUARE)
NEA_SHAPE(Triangle, WK_SHAPE_TRIANGLE)
NEA_SHAPE(Hexagon, WK_SHAPE_HEXAGON)
#undef NEA_SHAPE
}  // namespace RigidBodies
}  // namespace Objects

namespace Walker {
namespace PPO {
// Hyperparameters (Hyperparameters.cs:80-121): static-like defaults as a value type
struct Hyperparameters {
  wk_config c;
  Hyperparameters() { wk_config_defaults(&c); }
};
}  // namespace PPO
}  // namespace Walker

class Environment;

namespace Walker {
// Walker/Walker.cs surface for walker i of an Environment
class Walker {
 public:
  Walker(Environment* env, int index) : env_(env), i_(index) {}
  std::vector<float> GetState() const;                 // Walker.cs:132-152
  void TakeActions(const std::vector<float>& actions); // Walker.cs:66-75 (stored, applied by Update)
  std::pair<float, float> GetPosition() const;         // Walker.cs:108-111
  bool Terminal() const;
  wk_body_view Body(int part) const;                   // BodyParts (Walker.cs:237-245)
 private:
  Environment* env_;
  int i_;
};

namespace PPO {
// PPOAgent (Walker/PPO/PPOAgent.cs) over the context's device-resident networks
class PPOAgent {
 public:
  explicit PPOAgent(wk_ctx* ctx) : ctx_(ctx) {}
  // SampleActions (:381-398) for n states; env_ids/steps address the Philox noise
  void SampleActions(const std::vector<float>& states, std::vector<float>& actions,
                     std::vector<float>& logProbabilities, std::vector<float>& mean,
                     const std::vector<int32_t>& env_ids, const std::vector<uint32_t>& steps) {
    int n = (int)(states.size() / WK_OBS);
    actions.resize((size_t)n * WK_ACT);
    logProbabilities.resize((size_t)n * WK_ACT);
    mean.resize((size_t)n * WK_ACT);
    if (wk_policy_sample(ctx_, n, states.data(), env_ids.empty() ? nullptr : env_ids.data(),
                         steps.empty() ? nullptr : steps.data(), mean.data(), actions.data(),
                         logProbabilities.data()) != WK_OK)
      LogError(std::string("Exception thrown while attempting to sample actions: ") + wk_last_error(ctx_));
  }
  // GetValueEstimate (:350-364): 0 on failure, like the reference
  std::vector<float> GetValueEstimate(const std::vector<float>& states) {
    int n = (int)(states.size() / WK_OBS);
    std::vector<float> v((size_t)n, 0.0f);
    if (wk_value(ctx_, n, states.data(), v.data()) != WK_OK) {
      LogError(std::string("Exception thrown while attempting to get value estimate: ") + wk_last_error(ctx_));
      std::fill(v.begin(), v.end(), 0.0f);
    }
    return v;
  }
  // Train (:147-172) on the device trajectory; returns (critic, actor) diagnostics
  std::pair<float, float> Train(uint32_t update_index) {
    wk_ppo_args a{0, 0, 0, update_index};
    float cd = 0, ad = 0;
    if (wk_ppo_update(ctx_, &a, &cd, &ad) != WK_OK)
      LogError(std::string("Exception while training: ") + wk_last_error(ctx_));
    return {cd, ad};
  }
  std::vector<float> Save() {  // NeuralNetwork.Save order (flat)
    std::vector<float> p(WK_NPARAM);
    if (wk_get_weights(ctx_, p.data()) != WK_OK) LogError(wk_last_error(ctx_));
    return p;
  }
  void Load(const std::vector<float>& p) {
    if (p.size() != (size_t)WK_NPARAM) { LogError("Loading weights with the wrong size."); return; }
    if (wk_set_weights(ctx_, p.data()) != WK_OK) LogError(wk_last_error(ctx_));
  }
  // PPOAgent.Save (PPOAgent.cs:192-213): <filePath>Data/Weights/<critic|actor>.weights in
  // the reference's text format; the directory is created like Hyperparameters.CreateDirectories
  void Save(const std::string& filePath, const std::string& criticName = "critic",
            const std::string& actorName = "actor") {
    const std::string dir = filePath + "Data/Weights/";
    ::mkdir((filePath + "Data").c_str(), 0755);
    ::mkdir(dir.c_str(), 0755);
    if (wk_save_weights(ctx_, (dir + criticName + ".weights").c_str(),
                        (dir + actorName + ".weights").c_str()) != WK_OK)
      LogError(std::string("Exception while attempting to save the critic and actor neural networks: ") +
               wk_last_error(ctx_));
  }
  // NeuralNetwork.Load (NeuralNetwork.cs:94-115) for both networks from the same files
  void Load(const std::string& filePath, const std::string& criticName = "critic",
            const std::string& actorName = "actor") {
    const std::string dir = filePath + "Data/Weights/";
    if (wk_load_weights(ctx_, (dir + criticName + ".weights").c_str(),
                        (dir + actorName + ".weights").c_str()) != WK_OK)
      LogError(std::string("Loading neural network weights: ") + wk_last_error(ctx_));
  }
 private:
  wk_ctx* ctx_;
};
}  // namespace PPO
}  // namespace Walker

// Environment (Environment.cs) for N walkers on one GPU
class Environment {
 public:
  Environment(int n_walkers, const Walker::PPO::Hyperparameters& h = {}, uint64_t seed = 20250905,
              int device = 0, const Materials::IMaterial* material = nullptr)
      : n_(n_walkers) {
    if (wk_create(&h.c, device, n_walkers, seed, &ctx_) != WK_OK)
      throw std::runtime_error(std::string("wk_create: ") + wk_last_error(nullptr));
    if (material) {
      std::vector<int32_t> m((size_t)n_, material->Id());
      if (wk_set_materials(ctx_, m.data()) != WK_OK) LogError(wk_last_error(ctx_));
    }
    state_.assign((size_t)n_ * WK_OBS, 0.0f);
    pending_.clear();
    InitialState();
  }
  ~Environment() { wk_destroy(ctx_); }
  Environment(const Environment&) = delete;
  Environment& operator=(const Environment&) = delete;

  // Environment.Update (:64-92) for every walker: policy sampling (or the actions given
  // to Walker.TakeActions), physics, reward, terminal, auto-reset.  deltaTime must be
  // the fixed MonoGame step the context was created with (Game1.cs:60,73).
  void Update(float deltaTime) {
    if (deltaTime <= 0.0f) { LogError("Non-positive deltaTime."); return; }
    rewards_.assign((size_t)n_, 0.0f);
    dones_.assign((size_t)n_, 0);
    const float* a = pending_.empty() ? nullptr : pending_.data();
    if (wk_step(ctx_, a, 1, state_.data(), rewards_.data(), dones_.data(), nullptr) != WK_OK)
      LogError(std::string("Exception occurred during the environment update: ") + wk_last_error(ctx_));
    pending_.clear();
    steps_++;
  }
  // StepObjects with caller actions (clipped in-kernel like Environment.cs:78)
  void StepObjects(const std::vector<float>& actions) {
    pending_ = actions;
    Update(1.0f);
  }
  // _rigidBodies.Add(...) after CreateFloor() (Environment.cs:39-51) for every walker
  void AddRigidBodies(const std::vector<Objects::RigidBodies::Prop>& props) {
    std::vector<wk_prop> d;
    for (const auto& p : props) d.push_back(p.Desc());
    if (wk_set_scene(ctx_, d.data(), (int)d.size()) != WK_OK) LogError(wk_last_error(ctx_));
  }
  // InitialState (:176-180)
  void InitialState() {
    if (wk_get_obs(ctx_, state_.data()) != WK_OK) LogError(wk_last_error(ctx_));
  }
  // GetConsoleInformation (:56-60) for walker i: (episode, x position, state)
  std::tuple<int, float, std::vector<float>> GetConsoleInformation(int i) {
    wk_body_view b{};
    if (wk_get_body_view(ctx_, i, 2, &b) != WK_OK) LogError(wk_last_error(ctx_));
    std::vector<float> st(state_.begin() + (size_t)i * WK_OBS, state_.begin() + (size_t)(i + 1) * WK_OBS);
    std::vector<float> s((size_t)n_ * WK_STATE_FLOATS);
    int ep = 0;
    if (wk_get_state(ctx_, s.data()) == WK_OK) ep = (int)s[(size_t)i * WK_STATE_FLOATS + WK_ST_EPISODES];
    return {ep, b.centroid[0], st};
  }
  Walker::Walker GetWalker(int i) { return Walker::Walker(this, i); }
  Walker::PPO::PPOAgent Brain() { return Walker::PPO::PPOAgent(ctx_); }
  const std::vector<float>& State() const { return state_; }
  const std::vector<float>& Rewards() const { return rewards_; }
  const std::vector<uint8_t>& Dones() const { return dones_; }
  int Count() const { return n_; }
  wk_ctx* Context() { return ctx_; }

 private:
  friend class Walker::Walker;
  wk_ctx* ctx_ = nullptr;
  int n_ = 0;
  long steps_ = 0;
  std::vector<float> state_, rewards_, pending_;
  std::vector<uint8_t> dones_;
};

namespace Walker {
inline std::vector<float> Walker::GetState() const {
  return std::vector<float>(env_->state_.begin() + (size_t)i_ * WK_OBS,
                            env_->state_.begin() + (size_t)(i_ + 1) * WK_OBS);
}
inline void Walker::TakeActions(const std::vector<float>& actions) {
  if (actions.size() != (size_t)WK_ACT) return;  // Walker.cs:68: height != joints -> ignored
  if (env_->pending_.empty()) env_->pending_.assign((size_t)env_->n_ * WK_ACT, 0.0f);
  for (int j = 0; j < WK_ACT; j++) env_->pending_[(size_t)i_ * WK_ACT + j] = actions[j];
}
inline std::pair<float, float> Walker::GetPosition() const {
  wk_body_view b{};
  if (wk_get_body_view(env_->ctx_, i_, 2, &b) != WK_OK) LogError(wk_last_error(env_->ctx_));
  return {b.centroid[0], b.centroid[1]};
}
inline bool Walker::Terminal() const { return !env_->dones_.empty() && env_->dones_[(size_t)i_]; }
inline wk_body_view Walker::Body(int part) const {
  wk_body_view b{};
  if (wk_get_body_view(env_->ctx_, i_, part, &b) != WK_OK) LogError(wk_last_error(env_->ctx_));
  return b;
}
}  // namespace Walker

}  // namespace NEA
