// lzm_atari.h — device side of the collect loop for the Atari image configs (BASELINE.json config 5,
// Breakout MuZero).
//
// What the reference collector does per env step for an Atari env (lzero/worker/muzero_collector.py:
// 399-705 with zoo/atari/envs/atari_lightzero_env.py): select the action from the root visit counts
// (policy/utils.py:515-539), step the env, append the new grey 64x64 frame to the GameSegment
// (game_segment.py:129-149; the segment stores ONE frame per step and stacks frame_stack_num = 4 of
// them for the model, game_segment.py:95-127), store the search stats, and draw the next root's
// Dirichlet noise (policy/muzero.py:660-676). Here one 256-thread workgroup per env does all of it in
// one launch right after the search: thread 0 runs the action choice, the recording of the scalars
// and the game logic; the 256 threads render the 64x64 frame (16 pixels each, 16-byte stores),
// record the u8 frame into the episode slot and shift the model's [4][64][64] float observation stack.
//
// The Arcade Learning Environment is not installed (no ROM, no ale_py), so the game is a STAND-IN
// with Breakout's interface: the minimal action set {NOOP, FIRE, RIGHT, LEFT} (FIRE serves the ball; it is
// also served after 8 idle steps, so episodes end under any policy), grey 64x64 frames as
// the reference's wrappers produce (WarpFrame 64x64, grey, scaled to [0, 1]), 6 rows of bricks worth
// 1 / 4 / 7 points by row pair as ALE scores them (clipped to their sign, as the collector env's
// ClipRewardWrapper does), one life per episode (EpisodicLifeEnv, the collector setting), truncation
// at max_episode_steps. Env parity is unpinned; the data path — frame format,
// per-step recording, trajectory sizes — has the real shape. Random streams are Philox per
// (seed, env, step, purpose) as in lzm_collect.h.
//
// The second game (GAME = 1, config 3's Pong EfficientZero) is a stand-in with Pong's interface: the minimal
// action set {NOOP, FIRE, RIGHT, LEFT, RIGHTFIRE, LEFTFIRE} (RIGHT moves the agent's paddle up, LEFT down, as
// ALE's Pong), the agent's paddle on the right, a scripted opponent on the left that tracks the ball at a
// lower speed, a point (+1 / -1) when the ball passes a paddle, the serve after FIRE or kPgAutoServe idle
// steps, the episode over at 21 points for either side (or at max_episode_steps), rewards clipped to their
// sign (already -1 / 0 / +1), the score (eval_episode_return) the point difference. The collect kernel
// is the same for both games; the game functions are chosen by the template parameter.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_collect.h"

namespace lzm {

constexpr int kAtHW = 64;                   // frame side
constexpr int kAtPix = kAtHW * kAtHW;       // 4096 pixels per frame
constexpr int kAtStack = 4;                 // frame_stack_num (atari_muzero_config.py)
constexpr int kAtThreads = 256;             // one workgroup per env, 16 pixels per thread
constexpr int kAtBrickRows = 6, kAtBrickCols = 15, kAtBrickY0 = 8, kAtBrickH = 2, kAtBrickW = 4;
constexpr int kAtPaddleY = 58, kAtPaddleW = 8, kAtPaddleSpeed = 3;
constexpr int kAtWall = 2;                  // wall thickness (top, left, right)
constexpr int kAtSub = 2;                   // ball sub-steps per env step
constexpr int kAtStateWords = 16;
constexpr int kAtAutoServe = 8;             // idle steps before the ball is served without FIRE

// state words per env
// (AT_SCORE: the episode's unclipped points so far, the env's eval_episode_return)
enum { AT_PADDLE = 0, AT_BX, AT_BY, AT_VX, AT_VY, AT_IN_PLAY, AT_BRICK0, AT_BRICK1, AT_BRICK2, AT_LIVES, AT_IDLE, AT_SCORE };

struct AtariArgs {
  int n, A, T, E, max_steps, deterministic;
  float temperature, noise_alpha;
  uint32_t seed;
  const int64_t *counter;      // env-step counter (device)
  const int32_t *visits;       // [n][A] root visit counts (legal order)
  const float *root_value;     // [n]
  int32_t *state;              // [n][16]
  int32_t *steps;              // [n] steps taken in the current episode
  uint8_t *cur;                // [n][4096] the newest frame (u8)
  float *obs;                  // [n][4][64][64] the model's observation stack (frame / 255)
  float *noises;               // [n][A] next root's Dirichlet noise (out)
  uint8_t *rec_frames;         // [n][E][T+1][4096]
  int32_t *rec_action;         // [n][E][T]
  float *rec_reward;           // [n][E][T]
  int32_t *rec_visits;         // [n][E][T][A]
  float *rec_value;            // [n][E][T]
  const float *pred_value;     // [n] (nullable: priorities off)
  float *rec_pred;             // [n][E][T] (nullable)
  int32_t *ep_len;             // [n][E]
  int32_t *ep_count;           // [n]
  float *ep_return;            // [n][E] unclipped score of the finished episode in each slot (nullable)
};

__device__ inline bool at_brick(const int32_t *s, int r, int c) {
  const int b = r * kAtBrickCols + c;
  return ((uint32_t)s[AT_BRICK0 + (b >> 5)] >> (b & 31)) & 1u;
}

__device__ inline void at_reset(int32_t *s, PhiloxStream &rs) {
  const uint4 r = rs.next();
  for (int k = 0; k < kAtStateWords; ++k) s[k] = 0;
  s[AT_PADDLE] = kAtWall + (int)(r.x % (uint32_t)(kAtHW - 2 * kAtWall - kAtPaddleW + 1));
  s[AT_BRICK0] = -1;                                        // bricks 0..31
  s[AT_BRICK1] = -1;                                        // 32..63
  s[AT_BRICK2] = (1 << (kAtBrickRows * kAtBrickCols - 64)) - 1;  // 64..89
  s[AT_LIVES] = 1;
}

// One env step of the stand-in game: returns the reward; *terminated when the ball is lost.
__device__ inline float at_step(int32_t *s, int action, PhiloxStream &rs, bool *terminated) {
  *terminated = false;
  int px = s[AT_PADDLE];
  if (action == 2) px += kAtPaddleSpeed;
  if (action == 3) px -= kAtPaddleSpeed;
  px = px < kAtWall ? kAtWall : (px > kAtHW - kAtWall - kAtPaddleW ? kAtHW - kAtWall - kAtPaddleW : px);
  s[AT_PADDLE] = px;
  if (!s[AT_IN_PLAY]) {
    // served by FIRE, or after kAtAutoServe idle steps (a stand-in convenience: episodes end under any
    // policy, e.g. an untrained network that never picks FIRE)
    s[AT_IDLE] += 1;
    if (action != 1 && s[AT_IDLE] < kAtAutoServe) return 0.0f;
    s[AT_IDLE] = 0;
    const uint4 r = rs.next();
    s[AT_IN_PLAY] = 1;
    s[AT_BX] = px + kAtPaddleW / 2 - 1;
    s[AT_BY] = kAtPaddleY - 8;
    s[AT_VX] = (r.x & 1) ? 1 : -1;
    s[AT_VY] = -1;
    return 0.0f;
  }
  float reward = 0.0f;
  int x = s[AT_BX], y = s[AT_BY], vx = s[AT_VX], vy = s[AT_VY];
  for (int sub = 0; sub < kAtSub; ++sub) {
    int nx = x + vx, ny = y + vy;
    if (nx < kAtWall) { nx = kAtWall; vx = -vx; }
    if (nx > kAtHW - kAtWall - 2) { nx = kAtHW - kAtWall - 2; vx = -vx; }
    if (ny < kAtWall) { ny = kAtWall; vy = -vy; }
    // bricks: the first live brick under one of the ball's four pixels breaks; the ball turns back
    bool hit = false;
    for (int k = 0; k < 4 && !hit; ++k) {
      const int bx = nx + (k & 1), by = ny + (k >> 1);
      if (by < kAtBrickY0 || by >= kAtBrickY0 + kAtBrickRows * kAtBrickH || bx < kAtWall) continue;
      const int r = (by - kAtBrickY0) / kAtBrickH, c = (bx - kAtWall) / kAtBrickW;
      if (c >= kAtBrickCols || !at_brick(s, r, c)) continue;
      const int b = r * kAtBrickCols + c;
      s[AT_BRICK0 + (b >> 5)] &= (int32_t)~(1u << (b & 31));
      reward += r < 2 ? 7.0f : (r < 4 ? 4.0f : 1.0f);  // ALE Breakout: 7 / 4 / 1 points by row pair
      hit = true;
    }
    if (hit) { vy = -vy; ny = y; }
    // paddle
    if (vy > 0 && ny + 1 >= kAtPaddleY && ny <= kAtPaddleY + 1 && nx + 1 >= px && nx <= px + kAtPaddleW - 1) {
      const int off = (nx + 1) - (px + kAtPaddleW / 2);
      vx = off < -2 ? -2 : (off < 0 ? -1 : (off < 2 ? 1 : 2));
      vy = -vy;
      ny = kAtPaddleY - 2;
    }
    x = nx;
    y = ny;
    if (y > kAtHW - 2) {  // the ball is lost: one life per episode
      s[AT_IN_PLAY] = 0;
      s[AT_LIVES] -= 1;
      *terminated = s[AT_LIVES] <= 0;
      break;
    }
  }
  s[AT_BX] = x; s[AT_BY] = y; s[AT_VX] = vx; s[AT_VY] = vy;
  if (!s[AT_BRICK0] && !s[AT_BRICK1] && !s[AT_BRICK2]) {  // wall cleared: a fresh wall
    s[AT_BRICK0] = -1;
    s[AT_BRICK1] = -1;
    s[AT_BRICK2] = (1 << (kAtBrickRows * kAtBrickCols - 64)) - 1;
  }
  return reward;
}

// 16 consecutive pixels of row y from column x0 (thread tid renders y = tid / 4, x0 = 16 (tid % 4))
__device__ inline void at_render16(const int32_t *s, int tid, uint8_t px[16]) {
  const int y = tid >> 2, x0 = (tid & 3) * 16;
  const int pad = s[AT_PADDLE], bx = s[AT_BX], by = s[AT_BY], inp = s[AT_IN_PLAY];
  for (int j = 0; j < 16; ++j) {
    const int x = x0 + j;
    uint8_t v = 0;
    if (y < kAtWall || x < kAtWall || x >= kAtHW - kAtWall) {
      v = 142;
    } else if (y >= kAtBrickY0 && y < kAtBrickY0 + kAtBrickRows * kAtBrickH) {
      const int r = (y - kAtBrickY0) / kAtBrickH, c = (x - kAtWall) / kAtBrickW;
      if (c < kAtBrickCols && at_brick(s, r, c)) v = (uint8_t)(200 - 16 * r);
    }
    if (y >= kAtPaddleY && y < kAtPaddleY + 2 && x >= pad && x < pad + kAtPaddleW) v = 200;
    if (inp && x >= bx && x < bx + 2 && y >= by && y < by + 2) v = 236;
    px[j] = v;
  }
}

__device__ inline uint4 at_pack16(const uint8_t px[16]) {
  uint32_t w[4];
  for (int q = 0; q < 4; ++q)
    w[q] = (uint32_t)px[4 * q] | ((uint32_t)px[4 * q + 1] << 8) | ((uint32_t)px[4 * q + 2] << 16) |
           ((uint32_t)px[4 * q + 3] << 24);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// the stack's frames k: 16 floats of this thread's pixels
__device__ inline void at_store_obs16(float *obs_env, int k, int tid, const uint8_t px[16]) {
  float4 *dst = reinterpret_cast<float4 *>(obs_env + (size_t)k * kAtPix + tid * 16);
  const float sc = 1.0f / 255.0f;
  for (int q = 0; q < 4; ++q)
    dst[q] = make_float4(px[4 * q] * sc, px[4 * q + 1] * sc, px[4 * q + 2] * sc, px[4 * q + 3] * sc);
}

// ---- the Pong stand-in (GAME = 1)
constexpr int kPgPaddleH = 8, kPgSpeed = 3, kPgOppSpeed = 2, kPgMeX = 56, kPgOppX = 6, kPgAutoServe = 8, kPgWin = 21;
// state words (PG_SCORE at AT_SCORE's index: the collect kernel accumulates it)
enum { PG_PADDLE = 0, PG_BX, PG_BY, PG_VX, PG_VY, PG_IN_PLAY, PG_OPP, PG_ME_PTS, PG_OPP_PTS, PG_UNUSED, PG_IDLE,
       PG_SCORE };
static_assert(PG_SCORE == AT_SCORE, "score word");

__device__ inline void pg_reset(int32_t *s, PhiloxStream &rs) {
  const uint4 r = rs.next();
  for (int k = 0; k < kAtStateWords; ++k) s[k] = 0;
  const int span = kAtHW - 2 * kAtWall - kPgPaddleH + 1;
  s[PG_PADDLE] = kAtWall + (int)(r.x % (uint32_t)span);
  s[PG_OPP] = kAtWall + (int)(r.y % (uint32_t)span);
}

__device__ inline int pg_clamp_paddle(int y) {
  return y < kAtWall ? kAtWall : (y > kAtHW - kAtWall - kPgPaddleH ? kAtHW - kAtWall - kPgPaddleH : y);
}

// the ball's vertical speed after a paddle hit at offset off of the ball's centre from the paddle's
__device__ inline int pg_bounce_vy(int off) { return off < -2 ? -2 : (off < 0 ? -1 : (off < 2 ? 1 : 2)); }

// One env step of the Pong stand-in: returns the points (+1 agent, -1 opponent); *terminated at 21 points.
__device__ inline float pg_step(int32_t *s, int action, PhiloxStream &rs, bool *terminated) {
  *terminated = false;
  const bool up = action == 2 || action == 4, down = action == 3 || action == 5;
  const bool fire = action == 1 || action == 4 || action == 5;
  const int py = pg_clamp_paddle(s[PG_PADDLE] + (up ? -kPgSpeed : 0) + (down ? kPgSpeed : 0));
  s[PG_PADDLE] = py;
  if (!s[PG_IN_PLAY]) {
    s[PG_IDLE] += 1;
    if (!fire && s[PG_IDLE] < kPgAutoServe) return 0.0f;
    s[PG_IDLE] = 0;
    const uint4 r = rs.next();
    s[PG_IN_PLAY] = 1;
    s[PG_BX] = kAtHW / 2 - 1;
    s[PG_BY] = kAtHW / 2 - 1;
    s[PG_VX] = (r.x & 1) ? 1 : -1;
    s[PG_VY] = (r.x & 2) ? 1 : -1;
    return 0.0f;
  }
  float pts = 0.0f;
  int x = s[PG_BX], y = s[PG_BY], vx = s[PG_VX], vy = s[PG_VY], oy = s[PG_OPP];
  for (int sub = 0; sub < kAtSub; ++sub) {
    // the opponent tracks the ball's centre
    const int oc = oy + kPgPaddleH / 2, bc = y + 1;
    oy = pg_clamp_paddle(oy + (bc > oc + 1 ? kPgOppSpeed : (bc < oc - 1 ? -kPgOppSpeed : 0)));
    int nx = x + vx, ny = y + vy;
    if (ny < kAtWall) { ny = kAtWall; vy = -vy; }
    if (ny > kAtHW - kAtWall - 2) { ny = kAtHW - kAtWall - 2; vy = -vy; }
    if (vx > 0 && nx + 1 >= kPgMeX && nx <= kPgMeX + 1 && ny + 1 >= py && ny <= py + kPgPaddleH - 1) {
      vy = pg_bounce_vy((ny + 1) - (py + kPgPaddleH / 2));
      vx = -vx;
      nx = kPgMeX - 2;
    } else if (vx < 0 && nx <= kPgOppX + 1 && nx + 1 >= kPgOppX && ny + 1 >= oy && ny <= oy + kPgPaddleH - 1) {
      vy = pg_bounce_vy((ny + 1) - (oy + kPgPaddleH / 2));
      vx = -vx;
      nx = kPgOppX + 2;
    }
    x = nx;
    y = ny;
    if (x < 0 || x > kAtHW - 2) {  // a point: the ball passed a paddle
      const bool mine = x < 0;
      pts = mine ? 1.0f : -1.0f;
      s[mine ? PG_ME_PTS : PG_OPP_PTS] += 1;
      s[PG_IN_PLAY] = 0;
      *terminated = s[PG_ME_PTS] >= kPgWin || s[PG_OPP_PTS] >= kPgWin;
      break;
    }
  }
  s[PG_BX] = x; s[PG_BY] = y; s[PG_VX] = vx; s[PG_VY] = vy; s[PG_OPP] = oy;
  return pts;
}

__device__ inline void pg_render16(const int32_t *s, int tid, uint8_t px[16]) {
  const int y = tid >> 2, x0 = (tid & 3) * 16;
  const int py = s[PG_PADDLE], oy = s[PG_OPP], bx = s[PG_BX], by = s[PG_BY], inp = s[PG_IN_PLAY];
  for (int j = 0; j < 16; ++j) {
    const int x = x0 + j;
    uint8_t v = 87;  // court
    if (y < kAtWall || y >= kAtHW - kAtWall) v = 236;
    if (x >= kPgMeX && x < kPgMeX + 2 && y >= py && y < py + kPgPaddleH) v = 147;
    if (x >= kPgOppX && x < kPgOppX + 2 && y >= oy && y < oy + kPgPaddleH) v = 130;
    if (inp && x >= bx && x < bx + 2 && y >= by && y < by + 2) v = 236;
    px[j] = v;
  }
}

template <int GAME>
__device__ inline void game_reset(int32_t *s, PhiloxStream &rs) {
  if constexpr (GAME == 1) pg_reset(s, rs); else at_reset(s, rs);
}
template <int GAME>
__device__ inline float game_step(int32_t *s, int action, PhiloxStream &rs, bool *terminated) {
  if constexpr (GAME == 1) return pg_step(s, action, rs, terminated); else return at_step(s, action, rs, terminated);
}
template <int GAME>
__device__ inline void game_render16(const int32_t *s, int tid, uint8_t px[16]) {
  if constexpr (GAME == 1) pg_render16(s, tid, px); else at_render16(s, tid, px);
}

template <int GAME>
__global__ void __launch_bounds__(kAtThreads) atari_reset_kernel(int n, int32_t *state, int32_t *steps, uint8_t *cur,
                                                                 float *obs, uint32_t seed) {
  const int i = blockIdx.x, tid = threadIdx.x;
  __shared__ int32_t s[kAtStateWords];
  if (tid == 0) {
    PhiloxStream rs{seed, (uint32_t)i, 0xffffffffu, 0xffffffffu, 5u, 0u};
    game_reset<GAME>(s, rs);
    for (int k = 0; k < kAtStateWords; ++k) state[(size_t)i * kAtStateWords + k] = s[k];
    steps[i] = 0;
  }
  __syncthreads();
  uint8_t px[16];
  game_render16<GAME>(s, tid, px);
  reinterpret_cast<uint4 *>(cur + (size_t)i * kAtPix)[tid] = at_pack16(px);
  float *ob = obs + (size_t)i * kAtStack * kAtPix;
  for (int k = 0; k < kAtStack; ++k) at_store_obs16(ob, k, tid, px);  // the reset window: 4 x the first frame
}

template <int GAME>
__global__ void __launch_bounds__(kAtThreads) atari_collect_kernel(AtariArgs p) {
  const int i = blockIdx.x, tid = threadIdx.x;
  __shared__ int32_t s1[kAtStateWords], s0[kAtStateWords];
  __shared__ int sh_t, sh_done, sh_nt;
  __shared__ long long sh_slot;
  const uint64_t step = (uint64_t)*p.counter;
  const int A = p.A;
  if (tid == 0) {
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
    // ---- record the transition's scalars (GameSegment.append + store_search_stats)
    const int e = p.ep_count[i] % p.E;
    const int t = p.steps[i];
    const size_t slot = (size_t)i * p.E + e;
    if (t < p.T) {
      p.rec_action[slot * p.T + t] = action;
      for (int a = 0; a < A; ++a) p.rec_visits[(slot * p.T + t) * A + a] = v[a];
      p.rec_value[slot * p.T + t] = p.root_value[i];
      if (p.rec_pred) p.rec_pred[slot * p.T + t] = p.pred_value[i];
    }
    // ---- env step
    for (int k = 0; k < kAtStateWords; ++k) s1[k] = p.state[(size_t)i * kAtStateWords + k];
    PhiloxStream rg{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 6u, 0u};
    bool terminated = false;
    // ClipRewardWrapper (the collector env's clip_rewards=True, atari_lightzero_env.py:57): sign(points);
    // the unclipped points add up to the episode's return, the env's eval_episode_return
    const float points = game_step<GAME>(s1, action, rg, &terminated);
    s1[AT_SCORE] += (int32_t)points;
    const float reward = points > 0.0f ? 1.0f : (points < 0.0f ? -1.0f : 0.0f);
    const int nt = t + 1;
    const bool done = terminated || nt >= p.max_steps;
    if (t < p.T) p.rec_reward[slot * p.T + t] = reward;
    if (done) {
      p.ep_len[slot] = nt;
      if (p.ep_return) p.ep_return[slot] = (float)s1[AT_SCORE];
      p.ep_count[i] += 1;
      PhiloxStream rr{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 3u, 0u};
      game_reset<GAME>(s0, rr);
      p.steps[i] = 0;
      for (int k = 0; k < kAtStateWords; ++k) p.state[(size_t)i * kAtStateWords + k] = s0[k];
    } else {
      p.steps[i] = nt;
      for (int k = 0; k < kAtStateWords; ++k) p.state[(size_t)i * kAtStateWords + k] = s1[k];
    }
    sh_t = t;
    sh_nt = nt;
    sh_done = done ? 1 : 0;
    sh_slot = (long long)slot;
    // ---- next root's Dirichlet(alpha) noise
    PhiloxStream rn{p.seed, (uint32_t)i, (uint32_t)step, (uint32_t)(step >> 32), 4u, 0u};
    double g[64], gs = 0.0;
    for (int a = 0; a < A; ++a) {
      g[a] = gamma_sample((double)p.noise_alpha, rn);
      gs += g[a];
    }
    for (int a = 0; a < A; ++a) p.noises[(size_t)i * A + a] = (float)(gs > 0.0 ? g[a] / gs : 1.0 / A);
  }
  __syncthreads();
  const int t = sh_t, nt = sh_nt;
  const size_t slot = (size_t)sh_slot;
  uint4 *cur = reinterpret_cast<uint4 *>(p.cur + (size_t)i * kAtPix);
  uint4 *rec = reinterpret_cast<uint4 *>(p.rec_frames + slot * (size_t)(p.T + 1) * kAtPix);
  // the frame the search saw (o_t) into the episode slot
  if (t < p.T) rec[(size_t)t * (kAtPix / 16) + tid] = cur[tid];
  uint8_t px[16];
  game_render16<GAME>(s1, tid, px);  // o_{t+1}
  float *ob = p.obs + (size_t)i * kAtStack * kAtPix;
  if (!sh_done) {
    cur[tid] = at_pack16(px);
    // shift the stack by one frame (each thread moves its own pixels: no cross-thread hazard)
    float4 *o4 = reinterpret_cast<float4 *>(ob);
    for (int k = 0; k + 1 < kAtStack; ++k)
      for (int q = 0; q < 4; ++q)
        o4[(size_t)k * (kAtPix / 4) + tid * 4 + q] = o4[(size_t)(k + 1) * (kAtPix / 4) + tid * 4 + q];
    at_store_obs16(ob, kAtStack - 1, tid, px);
  } else {
    if (nt <= p.T) rec[(size_t)nt * (kAtPix / 16) + tid] = at_pack16(px);  // the episode's final frame
    game_render16<GAME>(s0, tid, px);  // the next episode's first frame
    cur[tid] = at_pack16(px);
    for (int k = 0; k < kAtStack; ++k) at_store_obs16(ob, k, tid, px);
  }
}

}  // namespace lzm
