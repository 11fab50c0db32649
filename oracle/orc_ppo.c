/*
 * orc_ppo.c -- CPU restatement of the reference's hand-rolled MLP, PPO and Adam.
 * TEST INFRASTRUCTURE ONLY (see wk_oracle.h).  PARITY UNPINNED (see wk_oracle.h).
 *
 * Follows:
 *   Walker/PPO/Matrix.cs           (operator* :180-199 with sequential Multiply :604-616,
 *                                   Clip :377-405, InRange :408-433, LessThan :436-461,
 *                                   LessThanNotEquals :464-489, Flatten :507-523,
 *                                   FromXavier :59-80, SampleNormal :541-555,
 *                                   LogNormalDensities :557-571, Average :588-602)
 *   Walker/PPO/NormalDistribution.cs (BoxMullerTransform :12-19, LogProbabilityDensity :24-32)
 *   Walker/PPO/Network/DenseLayer.cs (FeedForward :82-98, FeedBack :103-120, Adam :125-159)
 *   Walker/PPO/Network/ActivationLayer.cs (:12-73), NeuralNetwork.cs (:52-91, :179-185)
 *   Walker/PPO/PPOAgent.cs         (Train(Trajectory) :147-172, CalculateValues :175-189,
 *                                   Train(Batch) :218-346, SampleActions :381-398,
 *                                   GAE :414-444, Normalize :461-472, MC :475-498,
 *                                   CreateBatches :501-540)
 * Default networks (Hyperparameters.cs:91-92): critic 12-64-LReLU-1,
 * actor 12-64-LReLU-64-LReLU-4-TanH.  Flat parameter order: critic layers then actor
 * layers, each dense layer W (out x in, row-major) then B -- the .weights order
 * (DenseLayer.cs:73-79).
 */
#include "wk_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { L_DENSE = 0, L_RELU = 1, L_LRELU = 2, L_TANH = 3 };

typedef struct {
  int type, in, out;
  float *W, *b, *dW, *db, *mW, *mb, *vW, *vb;
  int iteration;
} layer;

typedef struct {
  int nl;
  layer L[8];
  float cache[8][64]; /* input of every layer (NeuralNetwork.cs:54-58) */
  int cache_n[8];
} net;

struct orc_agent {
  orc_hyper h;
  net critic, actor;
  float* store; /* params, grads, m, v contiguous blocks */
};

static inline float net_maxf(float x, float y) {
  if (x != y) { if (!isnan(x)) return y < x ? x : y; return x; }
  return signbit(y) ? x : y;
}

static float box_muller(float mean, float std, float u1, float u2) {
  /* NormalDistribution.cs:12-19 */
  const float PI_F = 3.14159265358979323846f;
  if (u1 == 0.0f) u1 = 1.0f;
  float z = sqrtf(-2.0f * logf(u1)) * sinf(2.0f * PI_F * u2);
  return mean + (std * z);
}

float orc_log_density(float mean, float std, float action) {
  /* NormalDistribution.cs:24-32 */
  const float PI_F = 3.14159265358979323846f;
  float fraction = (action - mean) / std;
  fraction *= fraction;
  fraction /= 2.0f;
  return -logf(std) - logf(sqrtf(2.0f * PI_F)) - fraction;
}

static void net_add(net* n, int type, int in, int out) {
  layer* l = &n->L[n->nl++];
  memset(l, 0, sizeof(*l));
  l->type = type;
  l->in = in;
  l->out = out;
}

/* assign storage: params block P, grads G, adam m M, adam v Vv (each ORC_NPARAM) */
static size_t net_bind(net* n, float* P, float* G, float* M, float* Vv, size_t off) {
  for (int i = 0; i < n->nl; i++) {
    layer* l = &n->L[i];
    if (l->type != L_DENSE) continue;
    size_t nw = (size_t)l->out * l->in;
    l->W = P + off; l->dW = G + off; l->mW = M + off; l->vW = Vv + off; off += nw;
    l->b = P + off; l->db = G + off; l->mb = M + off; l->vb = Vv + off; off += l->out;
  }
  return off;
}

/* NeuralNetwork.FeedForward (NeuralNetwork.cs:52-64) */
static void net_forward(net* n, const float* x, int nx, float* y, int cache) {
  float cur[64], nxt[64];
  int cn = nx;
  memcpy(cur, x, sizeof(float) * nx);
  for (int i = 0; i < n->nl; i++) {
    layer* l = &n->L[i];
    if (cache) {
      memcpy(n->cache[i], cur, sizeof(float) * cn);
      n->cache_n[i] = cn;
    }
    if (l->type == L_DENSE) {
      /* DenseLayer.FeedForward: result = W * x (sequential sums), result += b */
      for (int j = 0; j < l->out; j++) {
        float s = 0.0f;
        for (int k = 0; k < l->in; k++) s += l->W[j * l->in + k] * cur[k];
        nxt[j] = s + l->b[j];
      }
      cn = l->out;
    } else {
      for (int j = 0; j < cn; j++) {
        float v = cur[j];
        if (l->type == L_RELU) nxt[j] = net_maxf(0.0f, v);
        else if (l->type == L_LRELU) nxt[j] = net_maxf(0.2f * v, v);
        else nxt[j] = tanhf(v);
      }
    }
    memcpy(cur, nxt, sizeof(float) * cn);
  }
  memcpy(y, cur, sizeof(float) * cn);
}

/* NeuralNetwork.FeedBack (NeuralNetwork.cs:67-82) */
static void net_backward(net* n, const float* g_in, int ng) {
  float g[64], r[64];
  memcpy(g, g_in, sizeof(float) * ng);
  int gn = ng;
  for (int i = n->nl - 1; i >= 0; i--) {
    layer* l = &n->L[i];
    const float* x = n->cache[i];
    if (l->type == L_DENSE) {
      /* DenseLayer.FeedBack (:103-120) */
      for (int j = 0; j < l->out; j++) l->db[j] = l->db[j] + (0.0f + g[j]);
      for (int j = 0; j < l->out; j++)
        for (int k = 0; k < l->in; k++)
          l->dW[j * l->in + k] = l->dW[j * l->in + k] + (0.0f + g[j] * x[k]);
      for (int k = 0; k < l->in; k++) {
        float s = 0.0f;
        for (int j = 0; j < l->out; j++) s += l->W[j * l->in + k] * g[j];
        r[k] = s;
      }
      gn = l->in;
      memcpy(g, r, sizeof(float) * gn);
    } else {
      /* ActivationLayer.FeedBack (:18-21): g (.) f'(cached input) */
      for (int j = 0; j < gn; j++) {
        float v = x[j], d;
        if (l->type == L_RELU) d = v < 0.0f ? 0.0f : 1.0f;
        else if (l->type == L_LRELU) d = v < 0.0f ? 0.2f : 1.0f;
        else d = (1.0f - (tanhf(v) * tanhf(v)));
        g[j] = g[j] * d;
      }
    }
  }
}

/* DenseLayer.Adam (:125-159) */
static void layer_adam(layer* l, const orc_hyper* h) {
  l->iteration += 1;
  float c1 = 1.0f - h->Beta1, c2 = 1.0f - h->Beta2;
  float bc1 = (float)(1.0 - pow((double)h->Beta1, (double)l->iteration));
  float bc2 = (float)(1.0 - pow((double)h->Beta2, (double)l->iteration));
  int nw = l->out * l->in;
  for (int pass = 0; pass < 2; pass++) {
    int n = pass ? l->out : nw;
    float* w = pass ? l->b : l->W;
    float* g = pass ? l->db : l->dW;
    float* m = pass ? l->mb : l->mW;
    float* v = pass ? l->vb : l->vW;
    for (int i = 0; i < n; i++) {
      m[i] = (g[i] * c1) + (m[i] * h->Beta1);
      v[i] = (v[i] * h->Beta2) + ((g[i] * g[i]) * c2);
      float mh = m[i] / bc1;
      float vh = v[i] / bc2;
      float den = sqrtf(vh) + h->AdamEpsilon;
      w[i] = w[i] - ((mh / den) * h->Alpha);
    }
  }
}

static void net_zero(net* n) {
  for (int i = 0; i < n->nl; i++) {
    layer* l = &n->L[i];
    if (l->type != L_DENSE) continue;
    memset(l->dW, 0, sizeof(float) * l->out * l->in);
    memset(l->db, 0, sizeof(float) * l->out);
  }
}

static void net_optimise(net* n, const orc_hyper* h) {
  for (int i = 0; i < n->nl; i++)
    if (n->L[i].type == L_DENSE) layer_adam(&n->L[i], h);
}

orc_agent* orc_agent_create(const orc_hyper* h, uint64_t seed) {
  orc_agent* a = (orc_agent*)calloc(1, sizeof(orc_agent));
  a->h = *h;
  a->store = (float*)calloc((size_t)ORC_NPARAM * 4, sizeof(float));
  float *P = a->store, *G = P + ORC_NPARAM, *M = G + ORC_NPARAM, *Vv = M + ORC_NPARAM;
  net_add(&a->critic, L_DENSE, 12, 64);
  net_add(&a->critic, L_LRELU, 64, 64);
  net_add(&a->critic, L_DENSE, 64, 1);
  net_add(&a->actor, L_DENSE, 12, 64);
  net_add(&a->actor, L_LRELU, 64, 64);
  net_add(&a->actor, L_DENSE, 64, 64);
  net_add(&a->actor, L_LRELU, 64, 64);
  net_add(&a->actor, L_DENSE, 64, 4);
  net_add(&a->actor, L_TANH, 4, 4);
  size_t off = net_bind(&a->critic, P, G, M, Vv, 0);
  off = net_bind(&a->actor, P, G, M, Vv, off);
  /* Xavier-normal W, zero B (DenseLayer.cs:35-36, Matrix.FromXavier :59-80), Philox
   * stream per dense layer (global dense-layer index: critic 0,1; actor 2,3,4). */
  int li = 0;
  net* nets[2] = {&a->critic, &a->actor};
  for (int q = 0; q < 2; q++)
    for (int i = 0; i < nets[q]->nl; i++) {
      layer* l = &nets[q]->L[i];
      if (l->type != L_DENSE) continue;
      float std = sqrtf(2.0f / (float)(l->out + l->in));
      for (int k = 0; k < l->out * l->in; k++) {
        float u1, u2;
        orc_xavier_uniforms(seed, li, k, &u1, &u2);
        l->W[k] = box_muller(0.0f, std, u1, u2);
      }
      li++;
    }
  return a;
}

void orc_agent_destroy(orc_agent* a) {
  free(a->store);
  free(a);
}

void orc_agent_get_params(const orc_agent* a, float* p) {
  memcpy(p, a->store, sizeof(float) * ORC_NPARAM);
}
void orc_agent_set_params(orc_agent* a, const float* p) {
  memcpy(a->store, p, sizeof(float) * ORC_NPARAM);
}
void orc_agent_get_adam(const orc_agent* a, float* m, float* v, int* t) {
  memcpy(m, a->store + 2 * ORC_NPARAM, sizeof(float) * ORC_NPARAM);
  memcpy(v, a->store + 3 * ORC_NPARAM, sizeof(float) * ORC_NPARAM);
  *t = a->critic.L[0].iteration;
}
void orc_agent_set_adam(orc_agent* a, const float* m, const float* v, int t) {
  memcpy(a->store + 2 * ORC_NPARAM, m, sizeof(float) * ORC_NPARAM);
  memcpy(a->store + 3 * ORC_NPARAM, v, sizeof(float) * ORC_NPARAM);
  net* nets[2] = {&a->critic, &a->actor};
  for (int q = 0; q < 2; q++)
    for (int i = 0; i < nets[q]->nl; i++) nets[q]->L[i].iteration = t;
}

void orc_actor_mean(orc_agent* a, const float s[12], float mean[4]) {
  net_forward(&a->actor, s, 12, mean, 0);
}
float orc_critic_value(orc_agent* a, const float s[12]) {
  float v;
  net_forward(&a->critic, s, 12, &v, 0);
  return v;
}

/* PPOAgent.SampleActions (:381-398) with Philox noise */
void orc_sample_actions(orc_agent* a, const float s[12], uint64_t seed, int env, uint32_t t,
                        float act[4], float logp[4]) {
  float mean[4];
  orc_actor_mean(a, s, mean);
  float std = expf(a->h.LogStandardDeviation);
  for (int d = 0; d < 4; d++) {
    float u1, u2;
    orc_noise_uniforms(seed, env, t, d, &u1, &u2);
    act[d] = box_muller(mean[d], std, u1, u2);
  }
  for (int d = 0; d < 4; d++) logp[d] = orc_log_density(mean[d], std, act[d]);
}

/* PPOAgent.Train(Batch) (:218-346) */
int orc_train_batch(orc_agent* a, int B, float B_div, const float* states, const float* actions,
                    const float* logp_old, const float* returns, const float* adv,
                    float* critic_diag, float* actor_diag, float* grads_out, int apply_adam) {
  const orc_hyper* h = &a->h;
  net_zero(&a->actor);
  net_zero(&a->critic);
  float std = expf(h->LogStandardDeviation);
  float avgC = 0.0f, avgA = 0.0f;
  float upper = 1.0f + h->Epsilon, lower = 1.0f - h->Epsilon;
  int skipped = 0;
  for (int i = 0; i < B; i++) {
    const float* s = states + 12 * i;
    const float* act = actions + 4 * i;
    const float* lpo = logp_old + 4 * i;
    float A = adv[i];
    float V;
    net_forward(&a->critic, s, 12, &V, 1);
    float criticLoss = 2.0f * (V - returns[i]);
    float mean[4];
    net_forward(&a->actor, s, 12, mean, 1);
    float lp[4], ratio[4], lcd[4], actorLoss[4];
    int skip = 0;
    for (int d = 0; d < 4; d++) lp[d] = orc_log_density(mean[d], std, act[d]);
    for (int d = 0; d < 4; d++) ratio[d] = expf(lp[d] - lpo[d]);
    for (int d = 0; d < 4; d++) {
      float r = ratio[d];
      float cr = r >= upper ? upper : (r <= lower ? lower : r);
      float cra = cr * A, ra = r * A;
      float partA = (ra <= cra ? 1.0f : 0.0f) * A;
      float partB = (cra < ra ? 1.0f : 0.0f) * A;
      float partC = (r >= lower && r <= upper) ? 1.0f : 0.0f;
      float l = partA + (partB * partC);
      l = l * -1.0f;
      float eo = expf(lpo[d]);
      if (eo == 0.0f) skip = 1; /* Matrix.HadamardDivision throws (Matrix.cs:364-368) */
      lcd[d] = skip ? 0.0f : l / eo;
    }
    if (skip) {
      skipped++;
      continue;
    }
    float var = std * std;
    for (int d = 0; d < 4; d++) {
      float prob = expf(lp[d]);
      float frac = (act[d] - mean[d]) / var;
      float md = prob * frac;
      actorLoss[d] = md * lcd[d];
    }
    criticLoss /= B_div;
    for (int d = 0; d < 4; d++) actorLoss[d] = actorLoss[d] / B_div;
    avgC += criticLoss;
    float sum = 0.0f;
    for (int d = 0; d < 4; d++) sum += actorLoss[d];
    avgA += sum / 4.0f;
    net_backward(&a->critic, &criticLoss, 1);
    net_backward(&a->actor, actorLoss, 4);
  }
  if (grads_out) memcpy(grads_out, a->store + ORC_NPARAM, sizeof(float) * ORC_NPARAM);
  if (apply_adam) {
    net_optimise(&a->critic, h);
    net_optimise(&a->actor, h);
  }
  if (critic_diag) *critic_diag = avgC;
  if (actor_diag) *actor_diag = avgA;
  return skipped;
}

/* MonteCarloReturn + MonteCarloAdvantages (:475-498), batched with an episode mask:
 * done[t] != 0 ends an episode at t (the reference trajectory is one episode, whose last
 * transition is the terminal one, so the mask reproduces G_T = 0 exactly). */
void orc_returns_mc(int T, const float* r, const float* v, const uint8_t* done, float gamma,
                    float* ret, float* adv) {
  float disc = 0.0f;
  for (int i = T - 1; i >= 0; i--) {
    if (done && done[i]) disc = 0.0f;
    disc = r[i] + (disc * gamma);
    ret[i] = disc;
  }
  for (int i = 0; i < T; i++) adv[i] = ret[i] - v[i];
}

/* GeneralizedAdvantageEstimate + CalculateDelta (:414-444).  Reference quirk kept:
 * nextGae is never updated, so A_t = delta_t + (gamma*lambda)*0. */
void orc_returns_gae(int T, const float* r, const float* v, const uint8_t* done, float gamma,
                     float lambda, float* ret, float* adv) {
  float nextGae = 0.0f, nextValue = 0.0f;
  for (int i = T - 1; i >= 0; i--) {
    if (done && done[i]) nextValue = 0.0f;
    float cur = v[i];
    float delta = r[i] + (gamma * nextValue) - cur;
    nextValue = cur;
    float gae = delta + (gamma * lambda * nextGae);
    adv[i] = gae;
    ret[i] = gae + v[i];
  }
}

/* Normalize (:461-472): LINQ Average/Sum accumulate in double; divides by std + Epsilon */
void orc_normalize(int n, float* x, float eps_clip) {
  if (n == 0) return;
  double s = 0.0;
  for (int i = 0; i < n; i++) s += (double)x[i];
  float mean = (float)(s / (double)n);
  double ss = 0.0;
  for (int i = 0; i < n; i++) {
    double d = (double)(x[i] - mean);
    ss += d * d;
  }
  float std = (float)sqrt(ss / (double)n);
  for (int i = 0; i < n; i++) {
    x[i] -= mean;
    x[i] /= std + eps_clip;
  }
}

/* PPOAgent.Train(Trajectory) (PPOAgent.cs:147-172) on one episode of T steps: value
 * estimates (:447-456), returns / advantages (:175-189), then Epochs x floor(T / BatchSize)
 * minibatches drawn without replacement (CreateBatches :501-540, keyed permutation for the
 * unseeded Random), each Train(Batch) + Adam (:218-346). */
void orc_train_trajectory(orc_agent* ag, const orc_hyper* h, uint64_t seed, uint32_t update, int T,
                          const float* S, const float* Ac, const float* Lp, const float* R) {
  float* Vv = (float*)malloc(sizeof(float) * (T + 1));
  float* G = (float*)malloc(sizeof(float) * (T + 1));
  float* Ad = (float*)malloc(sizeof(float) * (T + 1));
  float* bS = (float*)malloc(sizeof(float) * 12 * h->BatchSize);
  float* bA = (float*)malloc(sizeof(float) * 4 * h->BatchSize);
  float* bL = (float*)malloc(sizeof(float) * 4 * h->BatchSize);
  float* bG = (float*)malloc(sizeof(float) * h->BatchSize);
  float* bAd = (float*)malloc(sizeof(float) * h->BatchSize);
  for (int i = 0; i < T; i++) Vv[i] = orc_critic_value(ag, S + 12 * i);
  if (h->UseGAE) orc_returns_gae(T, R, Vv, NULL, h->Gamma, h->Lambda, G, Ad);
  else orc_returns_mc(T, R, Vv, NULL, h->Gamma, G, Ad);
  if (h->NormalizeAdvantages) orc_normalize(T, Ad, h->Epsilon);
  int nb = T / h->BatchSize;
  for (int ep = 0; ep < h->Epochs; ep++) {
    uint32_t key[4];
    orc_perm_key(seed, update, (uint32_t)ep, key);
    for (int b = 0; b < nb; b++) {
      for (int k = 0; k < h->BatchSize; k++) {
        uint32_t idx = orc_perm((uint32_t)(b * h->BatchSize + k), (uint32_t)T, key);
        memcpy(bS + 12 * k, S + 12 * idx, sizeof(float) * 12);
        memcpy(bA + 4 * k, Ac + 4 * idx, sizeof(float) * 4);
        memcpy(bL + 4 * k, Lp + 4 * idx, sizeof(float) * 4);
        bG[k] = G[idx];
        bAd[k] = Ad[idx];
      }
      orc_train_batch(ag, h->BatchSize, (float)h->BatchSize, bS, bA, bL, bG, bAd, NULL, NULL,
                      NULL, 1);
    }
  }
  free(Vv); free(G); free(Ad);
  free(bS); free(bA); free(bL); free(bG); free(bAd);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Game1.Update x n_steps on one walker with Train at every terminal step: the
 * reference's own single-threaded loop (CPU baseline workload).  env selects the walker's
 * Philox streams (one walker per thread in the all-cores baseline). */
int orc_reference_loop_env(const orc_hyper* h, uint64_t seed, int env_id, int n_steps,
                           double* train_seconds) {
  orc_env* env = orc_env_create(h, 0.0f, ORC_MAT_CARPET);
  orc_agent* ag = orc_agent_create(h, seed);
  int cap = h->MaxTimesteps + 2;
  float* S = (float*)malloc(sizeof(float) * 12 * cap);
  float* Ac = (float*)malloc(sizeof(float) * 4 * cap);
  float* Lp = (float*)malloc(sizeof(float) * 4 * cap);
  float* R = (float*)malloc(sizeof(float) * cap);
  float state[12];
  orc_env_get_obs(env, state);
  int T = 0, episodes = 0;
  uint32_t gstep = 0, update = 0;
  double tt = 0.0;
  for (int it = 0; it < n_steps; it++) {
    memcpy(S + 12 * T, state, sizeof(state));
    orc_sample_actions(ag, state, seed, env_id, gstep++, Ac + 4 * T, Lp + 4 * T);
    float rew;
    int done;
    orc_env_step(env, Ac + 4 * T, state, &rew, &done, NULL);
    R[T] = rew;
    T++;
    if (done) {
      const double t0 = now_s();
      orc_train_trajectory(ag, h, seed, update, T, S, Ac, Lp, R);
      tt += now_s() - t0;
      update++;
      episodes++;
      T = 0;
    }
  }
  if (train_seconds) *train_seconds = tt;
  free(S); free(Ac); free(Lp); free(R);
  orc_agent_destroy(ag);
  orc_env_destroy(env);
  return episodes;
}

int orc_reference_loop(const orc_hyper* h, uint64_t seed, int n_steps, double* train_seconds) {
  return orc_reference_loop_env(h, seed, 0, n_steps, train_seconds);
}

/* Environment.Update without the agent (physics only, Environment.cs:126-143 + reward /
 * terminal / reset): one walker, uniform actions in [-1, 1] from Philox (BASELINE config 2's
 * synthetic actions); returns the number of episodes. */
int orc_physics_loop(const orc_hyper* h, uint64_t seed, int env_id, int n_steps) {
  orc_env* env = orc_env_create(h, orc_env_offset(seed, env_id), ORC_MAT_CARPET);
  float a[4], obs[12], rew;
  int done, episodes = 0;
  for (int t = 0; t < n_steps; t++) {
    orc_synth_action(seed, env_id, (uint32_t)t, a);
    orc_env_step(env, a, obs, &rew, &done, NULL);
    episodes += done;
  }
  orc_env_destroy(env);
  return episodes;
}

/* seconds for one Train(Trajectory) on a T-step episode (the reference trains once per
 * episode; T = 1001 is a full-length one): the trajectory is sampled by the agent on the
 * walker, continuing through resets so any T is available. */
double orc_train_episode_seconds(const orc_hyper* h, uint64_t seed, int T) {
  orc_env* env = orc_env_create(h, 0.0f, ORC_MAT_CARPET);
  orc_agent* ag = orc_agent_create(h, seed);
  float* S = (float*)malloc(sizeof(float) * 12 * T);
  float* Ac = (float*)malloc(sizeof(float) * 4 * T);
  float* Lp = (float*)malloc(sizeof(float) * 4 * T);
  float* R = (float*)malloc(sizeof(float) * T);
  float state[12];
  orc_env_get_obs(env, state);
  for (int t = 0; t < T; t++) {
    memcpy(S + 12 * t, state, sizeof(state));
    orc_sample_actions(ag, state, seed, 0, (uint32_t)t, Ac + 4 * t, Lp + 4 * t);
    int done;
    orc_env_step(env, Ac + 4 * t, state, &R[t], &done, NULL);
  }
  const double t0 = now_s();
  orc_train_trajectory(ag, h, seed, 0, T, S, Ac, Lp, R);
  const double dt = now_s() - t0;
  free(S); free(Ac); free(Lp); free(R);
  orc_agent_destroy(ag);
  orc_env_destroy(env);
  return dt;
}
