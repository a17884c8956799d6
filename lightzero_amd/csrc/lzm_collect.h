// lzm_collect.h — device side of the collect loop for CartPole-v0.
//
// One thread per env, one launch per env step, right after the search: select the action from the
// root visit counts (lzero/policy/utils.py:515-539 select_action), record the transition the way
// GameSegment.append / store_search_stats do (lzero/mcts/buffer/game_segment.py:129-149, :205-218),
// step the env, auto-reset finished episodes, and draw the next root's Dirichlet noise
// (policy/muzero.py:660-676 uses np.random.dirichlet(alpha * ones(A))).
//
// CartPole-v0 dynamics are gymnasium's classic-control equations (the reference env wraps
// gymnasium.make('CartPole-v0'), zoo/classic_control/cartpole/envs/cartpole_lightzero_env.py): Euler
// integration in float64, tau 0.02, force 10, gravity 9.8, cart 1.0, pole 0.1, half-length 0.5,
// terminated when |x| > 2.4 or |theta| > 12 deg, truncated at 200 steps, reward 1 per step, reset
// to U(-0.05, 0.05)^4; observations are the state cast to float32. gymnasium is not installed here:
// env parity is unpinned (restated equations; tests check them against a numpy restatement).
// The random streams (action sampling, resets, noise) are Philox per (seed, env, step, purpose),
// not numpy's: statistically equivalent, not bit-identical to the reference's host RNG.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_numerics.h"

namespace lzm {

struct CollectArgs {
  int n, A, T, E, max_steps, deterministic;
  float temperature, noise_alpha;
  uint32_t seed;
  const int64_t *counter;      // env-step counter (device; the collect step's search advances it before this reads it)
  const int32_t *visits;       // [n][A] root visit counts (legal order)
  const float *root_value;     // [n]
  double *state;               // [n][4]
  int32_t *steps;              // [n] steps taken in the current episode
  float *obs;                  // [n][4] current observation (in: this step's root; out: next root)
  float *noises;               // [n][A] next root's Dirichlet noise (out)
  float *rec_obs;              // [n][E][T+1][4]
  int32_t *rec_action;         // [n][E][T]
  float *rec_reward;           // [n][E][T]
  int32_t *rec_visits;         // [n][E][T][A] root visit counts (store_search_stats normalises on the host)
  float *rec_value;            // [n][E][T]
  const float *pred_value;     // [n] the root's predicted value (nullable: priorities off)
  float *rec_pred;             // [n][E][T] (nullable)
  int32_t *ep_len;             // [n][E] length of the finished episode in each slot
  int32_t *ep_count;           // [n] finished episodes (slot of the running one = ep_count % E)
  float *ep_return;            // [n][E] return of the finished episode in each slot (nullable)
};

// uniform in (0, 1) from one Philox output word (53-bit double from two words)
__device__ inline double u01(uint32_t a, uint32_t b) {
  const uint64_t m = ((uint64_t)(a >> 5) << 26) | (b >> 6);  // 53 bits
  return ((double)m + 0.5) * (1.0 / 9007199254740992.0);
}

struct PhiloxStream {
  uint32_t seed, env, step_lo, step_hi, purpose, ctr;
  __device__ uint4 next() {
    return philox4x32_10(make_uint4(env, step_lo, step_hi, (purpose << 16) | (ctr++ & 0xffff)),
                         make_uint2(seed, 0x434f4c4cu));
  }
};

// Gamma(alpha) for alpha > 0 (Marsaglia & Tsang; alpha < 1 by Gamma(alpha + 1) * U^(1 / alpha)).
__device__ inline double gamma_sample(double alpha, PhiloxStream &rs) {
  const double boost_a = alpha < 1.0 ? alpha + 1.0 : alpha;
  const double d = boost_a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  double g = d;
  for (int it = 0; it < 64; ++it) {
    const uint4 r = rs.next();
    const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);  // Box-Muller
    const double v0 = 1.0 + c * z;
    if (v0 <= 0.0) continue;
    const double v = v0 * v0 * v0;
    const uint4 r2 = rs.next();
    const double u = u01(r2.x, r2.y);
    if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) {
      g = d * v;
      break;
    }
  }
  if (alpha < 1.0) {
    const uint4 r = rs.next();
    g *= pow(u01(r.x, r.y), 1.0 / alpha);
  }
  return g;
}

__device__ inline void cartpole_reset(double *s, PhiloxStream &rs) {
  const uint4 a = rs.next(), b = rs.next();
  s[0] = -0.05 + 0.1 * u01(a.x, a.y);
  s[1] = -0.05 + 0.1 * u01(a.z, a.w);
  s[2] = -0.05 + 0.1 * u01(b.x, b.y);
  s[3] = -0.05 + 0.1 * u01(b.z, b.w);
}

// gymnasium CartPoleEnv.step (Euler); returns terminated
__device__ inline bool cartpole_physics(double *s, int action) {
  const double gravity = 9.8, masscart = 1.0, masspole = 0.1, total_mass = masspole + masscart, length = 0.5;
  const double polemass_length = masspole * length, force_mag = 10.0, tau = 0.02;
  const double theta_threshold = 12.0 * 2.0 * 3.141592653589793 / 360.0, x_threshold = 2.4;
  double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
  const double force = action == 1 ? force_mag : -force_mag;
  const double costheta = cos(theta), sintheta = sin(theta);
  const double temp = (force + polemass_length * theta_dot * theta_dot * sintheta) / total_mass;
  const double thetaacc =
      (gravity * sintheta - costheta * temp) / (length * (4.0 / 3.0 - masspole * costheta * costheta / total_mass));
  const double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
  x = x + tau * x_dot;
  x_dot = x_dot + tau * xacc;
  theta = theta + tau * theta_dot;
  theta_dot = theta_dot + tau * thetaacc;
  s[0] = x; s[1] = x_dot; s[2] = theta; s[3] = theta_dot;
  return x < -x_threshold || x > x_threshold || theta < -theta_threshold || theta > theta_threshold;
}

__global__ void cartpole_reset_kernel(int n, double *state, int32_t *steps, float *obs, uint32_t seed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  PhiloxStream rs{seed, (uint32_t)i, 0xffffffffu, 0xffffffffu, 1u, 0u};
  double *s = state + (size_t)i * 4;
  cartpole_reset(s, rs);
  steps[i] = 0;
  for (int j = 0; j < 4; ++j) obs[(size_t)i * 4 + j] = (float)s[j];
}

__global__ void cartpole_collect_kernel(CollectArgs p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const int A = p.A;
  const uint64_t step = (uint64_t)*p.counter;
  PhiloxStream rs{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 2u, 0u};
  // ---- select_action: p_a = v_a^(1/T) / sum (float64), sample, or argmax (first max)
  const int32_t *v = p.visits + (size_t)i * A;
  int action = 0;
  if (p.deterministic) {
    for (int a = 1; a < A; ++a)
      if (v[a] > v[action]) action = a;
  } else {
    double tot = 0.0;
    const double inv_t = 1.0 / (double)p.temperature;
    for (int a = 0; a < A; ++a) tot += pow((double)(v[a] > 0 ? v[a] : 0), inv_t);
    const uint4 r = rs.next();
    const double u = u01(r.x, r.y) * tot;
    double cum = 0.0;
    action = -1;
    for (int a = 0; a < A; ++a) {
      const double pa = pow((double)(v[a] > 0 ? v[a] : 0), inv_t);
      cum += pa;
      if (action < 0 && pa > 0.0 && u < cum) action = a;
    }
    if (action < 0) action = A - 1;
  }
  // ---- record the transition (GameSegment.append + store_search_stats)
  const int e = p.ep_count[i] % p.E;
  const int t = p.steps[i];
  const size_t slot = (size_t)i * p.E + e;
  float *ob = p.obs + (size_t)i * 4;
  if (t < p.T) {
    for (int j = 0; j < 4; ++j) p.rec_obs[(slot * (p.T + 1) + t) * 4 + j] = ob[j];
    p.rec_action[slot * p.T + t] = action;
    for (int a = 0; a < A; ++a) p.rec_visits[(slot * p.T + t) * A + a] = v[a];
    p.rec_value[slot * p.T + t] = p.root_value[i];
    if (p.rec_pred) p.rec_pred[slot * p.T + t] = p.pred_value[i];
  }
  // ---- env step
  double *s = p.state + (size_t)i * 4;
  const bool terminated = cartpole_physics(s, action);
  const int nt = t + 1;
  const bool done = terminated || nt >= p.max_steps;
  if (t < p.T) p.rec_reward[slot * p.T + t] = 1.0f;
  if (done) {
    if (nt <= p.T)
      for (int j = 0; j < 4; ++j) p.rec_obs[(slot * (p.T + 1) + nt) * 4 + j] = (float)s[j];
    p.ep_len[slot] = nt;
    // eval_episode_return (cartpole_lightzero_env.py: the sum of the env's rewards, 1 per step)
    if (p.ep_return) p.ep_return[slot] = (float)nt;
    p.ep_count[i] += 1;
    PhiloxStream rr{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 3u, 0u};
    cartpole_reset(s, rr);
    p.steps[i] = 0;
  } else {
    p.steps[i] = nt;
  }
  for (int j = 0; j < 4; ++j) ob[j] = (float)s[j];
  // ---- next root's Dirichlet(alpha) noise
  PhiloxStream rn{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 4u, 0u};
  double g[64], gs = 0.0;
  for (int a = 0; a < A; ++a) {
    g[a] = gamma_sample((double)p.noise_alpha, rn);
    gs += g[a];
  }
  for (int a = 0; a < A; ++a) p.noises[(size_t)i * A + a] = (float)(gs > 0.0 ? g[a] / gs : 1.0 / A);
}

}  // namespace lzm
