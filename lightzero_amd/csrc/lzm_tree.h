// lzm_tree.h — device-side tree semantics shared by every tree kernel (gfx950).
//
// One restatement of LightZero's ctree node rules (reference paths under /root/reference):
// selection walk cbatch_traverse / compute_mean_q / cselect_child / cucb_score
// (lzero/mcts/ctree/ctree_muzero/lib/cnode.cpp:169-203, :551-596, :655-699, :755-824),
// CNode::expand (:83-147), cbackpropagate (:419-478) and the EfficientZero value-prefix
// variants (ctree_efficientzero/lib/cnode.cpp:173-212, :482-575, :756-814).
//
// TreeView addresses nodes as stat/meta[node * B + i]: over the whole batch in HBM (B = roots,
// i = root) or over a workgroup's slice staged in LDS (B = slice width, i = local root).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_numerics.h"

namespace lzm {

constexpr float kFloatMax = 1000000.0f;  // common_lib/cminimax.h:9-10
constexpr float kFloatMin = -kFloatMax;
constexpr int kMaxActions = 64;          // tie lists are held as one 64-bit mask
constexpr int kMaxWG = 1024;

struct alignas(16) NodeStat {
  int visit;
  float value_sum;
  float prior;
  float reward;  // value_prefix for EfficientZero
};
struct alignas(16) NodeMeta {
  int latent;  // current_latent_state_index, -1 while not expanded
  int to_play;
  int best;  // best_action
  int is_reset;
};

struct TreeView {
  NodeStat *stat;
  NodeMeta *meta;
  const int32_t *legal;   // [B][A]
  const int32_t *nlegal;  // [B]
  int32_t *path;          // [D][B] node ids
  int32_t *path_act;      // [D][B] actions
  int32_t *pathlen;       // [B] edges of the last path
  const float2 *lut;      // [N] {log((N+base+1)/base)+init, sqrt(N)}
  int B, A, cap, lut_n, depth_cap;
  // optional caches (the fused search keeps them in LDS; null elsewhere), bit-identical to the
  // divisions they replace: val[node * B + i] = node_value(stat) kept current by expand/backup;
  // pbt[N * (N + 1) / 2 + v] = lut[N].y / (v + 1) for child visits v <= N.
  float *val = nullptr;
  const float *pbt = nullptr;
};

__device__ inline size_t nidx(const TreeView &t, int node, int i) { return (size_t)node * t.B + i; }
__device__ inline float node_value(const NodeStat &s) {  // CNode::value, cnode.cpp:219-235
  return s.visit == 0 ? 0.0f : s.value_sum / (float)s.visit;
}
__device__ inline int legal_at(const TreeView &t, int i, int node, int j) {
  return node == 0 ? t.legal[(size_t)i * t.A + j] : j;
}
__device__ inline int legal_n(const TreeView &t, int i, int node) { return node == 0 ? t.nlegal[i] : t.A; }

// CMinMaxStats::normalize, common_lib/cminimax.cpp:33-45
__device__ inline float mm_normalize(float4 mm, float v) {
  float norm = v;
  float delta = mm.x - mm.y;
  if (delta > 0) {
    if (delta < mm.z)
      norm = (norm - mm.y) / mm.z;
    else
      norm = (norm - mm.y) / delta;
  }
  return norm;
}

// Result of one root's descent.
struct Descent {
  int len, x, action, vtp, leaf;
};

// One root's selection walk (cbatch_traverse body, cnode.cpp:783-823 with compute_mean_q
// :169-203, cselect_child :551-596, cucb_score :655-699; EZ variants
// ctree_efficientzero/lib/cnode.cpp:173-212, :756-814). `draw(level)` returns the rand()
// value consumed at that level. Writes path/path_act; never writes tree state.
// Tie information of a draw-free classification walk (descend with CLASSIFY = true).
struct TieInfo {
  int status;  // 0: walk complete, no tie; 1: stopped at a tie among unexpanded children (depth
               // known, child pending a draw); 2: stopped at a tie involving an expanded child
  int level;
  unsigned long long mask;  // tie candidates as legal positions
};

// i indexes the tree (stat/meta[node * t.B + i]); li / ps index the path arrays
// (path[level * ps + li]), which may live in LDS while the tree stays in HBM.
// CLASSIFY: stop at the first tie with more than one candidate and report it in `tie` instead
// of consuming a draw (forced levels still count as one draw each, like the reference).
template <bool EZ, bool CLASSIFY, typename Draw>
__device__ inline Descent descend_slice(const TreeView &t, int i, int li, int ps, float4 mm, int players, int vtp,
                                        float disc, Draw draw, TieInfo *tie) {
  int node = 0, is_root = 1, len = 0, last_action = -1, parent = 0;
  float parent_q = 0.0f;  // per root; the reference's cross-root carry is provably 0 wherever read
  NodeStat s = t.stat[nidx(t, 0, i)];
  NodeMeta m = t.meta[nidx(t, 0, i)];
  t.path[li] = 0;
  if (CLASSIFY) tie->status = 0;
  while (m.latent >= 0 && len < t.depth_cap - 1) {
    const int n = legal_n(t, i, node);
    const int base = 1 + t.A * m.latent;
    const float pvp = s.reward;
    const int preset = m.is_reset;
    // compute_mean_q
    float total_q = 0.0f;
    int total_v = 0;
    for (int j = 0; j < n; ++j) {
      const int a = legal_at(t, i, node, j);
      const NodeStat c = t.stat[nidx(t, base + a, i)];
      if (c.visit > 0) {
        float tr = c.reward;
        if (EZ) tr = preset == 1 ? c.reward : c.reward - pvp;
        const float cv = t.val ? t.val[nidx(t, base + a, i)] : node_value(c);
        float qsa = tr + disc * cv;
        total_q += qsa;
        total_v += 1;
      }
    }
    float mean_q;
    if (is_root && total_v > 0)
      mean_q = total_q / (float)total_v;
    else
      mean_q = (parent_q + total_q) / (float)(total_v + 1);
    is_root = 0;
    parent_q = mean_q;
    // cselect_child / cucb_score
    int N = s.visit - 1;
    N = N < 0 ? 0 : (N >= t.lut_n ? t.lut_n - 1 : N);
    const float2 L = t.lut[N];
    float max_score = kFloatMin;
    uint64_t mask = 0;
    for (int j = 0; j < n; ++j) {
      const int a = legal_at(t, i, node, j);
      const NodeStat c = t.stat[nidx(t, base + a, i)];
      float pb_c = L.x;
      pb_c *= (t.pbt && c.visit <= N) ? t.pbt[N * (N + 1) / 2 + c.visit] : (L.y / (float)(c.visit + 1));
      const float prior_score = pb_c * c.prior;
      float vs;
      if (c.visit == 0) {
        vs = mean_q;
      } else {
        float tr = c.reward;
        if (EZ) tr = preset == 1 ? c.reward : c.reward - pvp;
        const float cv = t.val ? t.val[nidx(t, base + a, i)] : node_value(c);
        if (players == 1)
          vs = tr + disc * cv;
        else
          vs = tr + disc * (-cv);
      }
      vs = mm_normalize(mm, vs);
      if (vs < 0) vs = 0;
      if (vs > 1) vs = 1;
      const float score = prior_score + vs;
      if (max_score < score) {
        max_score = score;
        mask = 1ull << j;
      } else if (score >= max_score - 0.000001f) {
        mask |= 1ull << j;
      }
    }
    const int nl = __popcll(mask);
    if (CLASSIFY && nl > 1) {
      bool all_leaves = true;
      for (uint64_t q = mask; q; q &= q - 1) {
        const int a = legal_at(t, i, node, __ffsll((long long)q) - 1);
        if (t.meta[nidx(t, base + a, i)].latent >= 0) all_leaves = false;
      }
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = mask;
      Descent d;
      d.len = len + 1;
      d.x = m.latent;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    const uint32_t r = CLASSIFY ? 0u : draw(len);
    int k = (int)(r % (uint32_t)nl);
    uint64_t mm_ = mask;
    for (; k > 0; --k) mm_ &= mm_ - 1;
    const int jsel = __ffsll((long long)mm_) - 1;
    const int action = legal_at(t, i, node, jsel);
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    t.path_act[(size_t)len * ps + li] = action;
    parent = node;
    node = base + action;
    last_action = action;
    ++len;
    t.path[(size_t)len * ps + li] = node;
    s = t.stat[nidx(t, node, i)];
    m = t.meta[nidx(t, node, i)];
  }
  Descent d;
  d.len = len;
  d.x = t.meta[nidx(t, parent, i)].latent;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

template <bool EZ, typename Draw>
__device__ inline Descent descend(const TreeView &t, int i, float4 mm, int players, int vtp, float disc, Draw draw) {
  return descend_slice<EZ, false>(t, i, i, t.B, mm, players, vtp, disc, draw, nullptr);
}

// DPP lane exchange inside a row of 16 lanes.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// The value of lane (lane ^ D) for a wave-wide xor butterfly step, without the LDS crossbar
// (__shfl_xor is a ds_bpermute: a dependent LDS round trip per step): D = 1, 2 quad_perm DPP; 4 two
// row shifts (row_shl:4 reads lane + 4, row_shr:4 lane - 4); 8 row_ror:8; 16, 32 the gfx950
// permlane swaps (with both operands v, each lane holds itself and its partner). The same pairs as
// __shfl_xor(v, D, 64), so a butterfly reduction built on it gives the same bits (measured: the
// Breakout / Pong one-launch searches +1% / +3% from their decodes).
template <int D>
__device__ __forceinline__ int xor_partner(int v) {
  const int lane = threadIdx.x & 63;
  if constexpr (D == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);
  } else if constexpr (D == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);
  } else if constexpr (D == 4) {
    const int up = __builtin_amdgcn_update_dpp(0, v, 0x104, 0xF, 0xF, false);
    const int dn = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    return (lane & 4) ? dn : up;
  } else if constexpr (D == 8) {
    return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);
  } else if constexpr (D == 16) {
    const auto pr = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane & 16) ? pr[0] : pr[1]);
  } else {
    static_assert(D == 32, "xor step");
    const auto pr = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane & 32) ? pr[0] : pr[1]);
  }
}
template <int D>
__device__ __forceinline__ float xor_partner(float v) {
  return __int_as_float(xor_partner<D>(__float_as_int(v)));
}
// sum / max over the wave in __shfl_xor butterfly order d = 32, 16, .., 1 (same bits); every lane
// of the wave must be active
template <typename T>
__device__ __forceinline__ T xor_sum(T v) {
  v += xor_partner<32>(v);
  v += xor_partner<16>(v);
  v += xor_partner<8>(v);
  v += xor_partner<4>(v);
  v += xor_partner<2>(v);
  v += xor_partner<1>(v);
  return v;
}
__device__ __forceinline__ float xor_max(float v) {
  v = fmaxf(v, xor_partner<32>(v));
  v = fmaxf(v, xor_partner<16>(v));
  v = fmaxf(v, xor_partner<8>(v));
  v = fmaxf(v, xor_partner<4>(v));
  v = fmaxf(v, xor_partner<2>(v));
  v = fmaxf(v, xor_partner<1>(v));
  return v;
}
__device__ __forceinline__ int xor_max(int v) {
  v = max(v, xor_partner<32>(v));
  v = max(v, xor_partner<16>(v));
  v = max(v, xor_partner<8>(v));
  v = max(v, xor_partner<4>(v));
  v = max(v, xor_partner<2>(v));
  v = max(v, xor_partner<1>(v));
  return v;
}
// sum and max together (independent chains interleaved)
__device__ __forceinline__ void xor_sum_max(float &s, float &m) {
#define LZM_XOR_STEP(D)                 \
  s += xor_partner<D>(s);               \
  m = fmaxf(m, xor_partner<D>(m));
  LZM_XOR_STEP(32) LZM_XOR_STEP(16) LZM_XOR_STEP(8) LZM_XOR_STEP(4) LZM_XOR_STEP(2) LZM_XOR_STEP(1)
#undef LZM_XOR_STEP
}
// max over the wave (rows of 16 by DPP, then the four row results by readlane)
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

// descend_slice with one whole wave per root, lane j scoring child j (legal position j), so a
// level costs one round of child reads instead of a serial chain. Bit-identical to the serial
// walk: the visited-children sum of compute_mean_q runs in child order (readlane loop), and the
// order-dependent tie list of cselect_child (running max, reset on a strictly larger score, append
// within 1e-6 of the running max) equals {r} + {j > r : score_j >= M - 1e-6}, where M is the
// maximum score and r its first position: the running max only ever resets at the first position
// reaching a new maximum, so the last reset is at r and from then on the running max is M.
// Every lane returns the same Descent; lane 0 writes the path. All 64 lanes must call it.
// true_action >= 0: ReZero search-with-reuse at the root (cbatch_traverse_with_reuse,
// ctree_muzero/lib/cnode.cpp:827-927): the true action's child is scored by carm_score (:702-749:
// its value term uses reuse_value instead of the child's value, and a visited child scores the
// value term alone), and choosing it ends the walk there even if the child is expanded (x = -1).
// RL: take the chosen child's records from the lane that read them (readlane) instead of re-reading
// them — for trees in global memory, where every dependent round of reads pays an L2-miss latency.
template <bool EZ, bool CLASSIFY, bool RL = false, typename Draw>
__device__ inline Descent descend_wave(const TreeView &t, int i, int li, int ps, float4 mm, int players, int vtp,
                                       float disc, Draw draw, TieInfo *tie, int true_action = -1,
                                       float reuse_value = 0.0f) {
  const int lane = threadIdx.x & 63;
  bool reuse_stop = false;
  int node = 0, is_root = 1, len = 0, last_action = -1, parent = 0;
  float parent_q = 0.0f;
  NodeStat s = t.stat[nidx(t, 0, i)];
  NodeMeta m = t.meta[nidx(t, 0, i)];
  if (lane == 0) t.path[li] = 0;
  if (CLASSIFY) tie->status = 0;
  while (m.latent >= 0 && len < t.depth_cap - 1) {
    const int n = legal_n(t, i, node);
    const int base = 1 + t.A * m.latent;
    const float pvp = s.reward;
    const int preset = m.is_reset;
    const bool valid = lane < n;
    const int a = valid ? legal_at(t, i, node, lane) : 0;
    // RL: every child's stat AND meta in one round of reads
    NodeStat c;
    NodeMeta cm;
    float cv = 0.0f;
    if (valid) {
      c = t.stat[nidx(t, base + a, i)];
      if (RL) cm = t.meta[nidx(t, base + a, i)];
      cv = t.val ? t.val[nidx(t, base + a, i)] : node_value(c);
    } else {
      c.visit = 0; c.value_sum = 0.0f; c.prior = 0.0f; c.reward = 0.0f;
      cm.latent = -1; cm.to_play = 0; cm.best = 0; cm.is_reset = 0;
    }
    float tr = c.reward;
    if (EZ) tr = preset == 1 ? c.reward : c.reward - pvp;
    // compute_mean_q: visited children in legal order
    const float qsa = tr + disc * cv;
    uint64_t vis = __ballot(valid && c.visit > 0);
    float total_q = 0.0f;
    const int total_v = __popcll(vis);
    for (uint64_t q = vis; q; q &= q - 1) total_q += readlane_f(qsa, __ffsll((long long)q) - 1);
    float mean_q;
    if (is_root && total_v > 0)
      mean_q = total_q / (float)total_v;
    else
      mean_q = (parent_q + total_q) / (float)(total_v + 1);
    is_root = 0;
    parent_q = mean_q;
    // cselect_child / cucb_score, every child at once
    int N = s.visit - 1;
    N = N < 0 ? 0 : (N >= t.lut_n ? t.lut_n - 1 : N);
    const float2 L = t.lut[N];
    float pb_c = L.x;
    pb_c *= (t.pbt && c.visit <= N) ? t.pbt[N * (N + 1) / 2 + c.visit] : (L.y / (float)(c.visit + 1));
    const float prior_score = pb_c * c.prior;
    const bool arm = len == 0 && true_action >= 0 && a == true_action;  // carm_score at the root
    const float cq = arm ? reuse_value : cv;
    float vs;
    if (c.visit == 0)
      vs = mean_q;
    else
      vs = (players == 1) ? tr + disc * cq : tr + disc * (-cq);
    vs = mm_normalize(mm, vs);
    if (vs < 0) vs = 0;
    if (vs > 1) vs = 1;
    const float score = (arm && c.visit > 0) ? vs : prior_score + vs;
    const float M = wave_max_dpp(valid ? score : -INFINITY);
    const int r = __ffsll((long long)__ballot(valid && score == M)) - 1;
    const uint64_t mask = __ballot(valid && lane > r && score >= M - 0.000001f) | (1ull << r);
    const int nl = __popcll(mask);
    if (CLASSIFY && nl > 1) {
      const bool leaf_child = !((mask >> lane) & 1ull) || (RL ? cm.latent : t.meta[nidx(t, base + a, i)].latent) < 0;
      const bool all_leaves = __ballot(!leaf_child) == 0ull;
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = mask;
      Descent d;
      d.len = len + 1;
      d.x = m.latent;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    const uint32_t rr = CLASSIFY ? 0u : draw(len);
    int k = (int)(rr % (uint32_t)nl);
    uint64_t mm_ = mask;
    for (; k > 0; --k) mm_ &= mm_ - 1;
    const int jsel = __ffsll((long long)mm_) - 1;
    const int action = __builtin_amdgcn_readlane(a, jsel);
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    parent = node;
    node = base + action;
    last_action = action;
    if (lane == 0) {
      t.path_act[(size_t)len * ps + li] = action;
      t.path[(size_t)(len + 1) * ps + li] = node;
    }
    ++len;
    if (RL) {
      s.visit = __builtin_amdgcn_readlane(c.visit, jsel);
      s.value_sum = readlane_f(c.value_sum, jsel);
      s.prior = readlane_f(c.prior, jsel);
      s.reward = readlane_f(c.reward, jsel);
      m.latent = __builtin_amdgcn_readlane(cm.latent, jsel);
      m.to_play = __builtin_amdgcn_readlane(cm.to_play, jsel);
      m.best = __builtin_amdgcn_readlane(cm.best, jsel);
      m.is_reset = __builtin_amdgcn_readlane(cm.is_reset, jsel);
    } else {
      s = t.stat[nidx(t, node, i)];
      m = t.meta[nidx(t, node, i)];
    }
    if (len == 1 && true_action >= 0 && action == true_action) {
      reuse_stop = true;  // cnode.cpp:888-891
      break;
    }
  }
  Descent d;
  d.len = len;
  d.x = (reuse_stop && m.latent >= 0) ? -1 : t.meta[nidx(t, parent, i)].latent;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}


// CNode::expand of a non-root leaf (cnode.cpp:83-147): all A actions legal, masked-softmax
// priors with glibc expf, sequential sum; children reset to CNode(prior, {}).
__device__ inline void expand_leaf(const TreeView &t, int i, int leaf, int to_play, int latent, float reward,
                                   const float *logits, int is_reset, bool ez) {
  NodeMeta m = t.meta[nidx(t, leaf, i)];
  m.latent = latent;
  m.to_play = to_play;
  if (ez) m.is_reset = is_reset;
  t.meta[nidx(t, leaf, i)] = m;
  t.stat[nidx(t, leaf, i)].reward = reward;
  float pmax = kFloatMin;
  for (int a = 0; a < t.A; ++a)
    if (pmax < logits[a]) pmax = logits[a];
  float sum = 0.0f;
  for (int a = 0; a < t.A; ++a) sum += glibc_expf(logits[a] - pmax);
  const int base = 1 + t.A * latent;
  for (int a = 0; a < t.A; ++a) {
    const float e = glibc_expf(logits[a] - pmax);
    NodeStat c;
    c.visit = 0;
    c.value_sum = 0.0f;
    c.prior = e / sum;
    c.reward = 0.0f;
    t.stat[nidx(t, base + a, i)] = c;
    NodeMeta cm;
    cm.latent = -1;
    cm.to_play = 0;
    cm.best = -1;
    cm.is_reset = 0;
    t.meta[nidx(t, base + a, i)] = cm;
    if (t.val) t.val[nidx(t, base + a, i)] = 0.0f;
  }
}

// cbackpropagate: MuZero cnode.cpp:419-478, EfficientZero
// ctree_efficientzero/lib/cnode.cpp:482-575.
template <bool EZ>
__device__ inline void backup_slice(const TreeView &t, int i, int li, int ps, float4 *mm_ptr, int to_play,
                                    float value, float disc) {
  float4 mm = *mm_ptr;
  const int len = t.pathlen[li];
  float b = value;
  for (int l = len; l >= 0; --l) {
    const int node = t.path[(size_t)l * ps + li];
    NodeStat s = t.stat[nidx(t, node, i)];
    const int ntp = t.meta[nidx(t, node, i)].to_play;
    if (to_play == -1 || ntp == to_play)
      s.value_sum += b;
    else
      s.value_sum += -b;
    s.visit += 1;
    t.stat[nidx(t, node, i)] = s;
    const float v = node_value(s);
    if (t.val) t.val[nidx(t, node, i)] = v;
    if (!EZ) {
      const float tr = s.reward;
      float q;
      if (to_play == -1) {
        q = tr + disc * v;
        b = tr + disc * b;
      } else {
        q = tr + disc * -v;
        b = (ntp == to_play) ? (-tr + disc * b) : (tr + disc * b);
      }
      if (q > mm.x) mm.x = q;
      if (q < mm.y) mm.y = q;
    } else {
      float pvp = 0.0f;
      int reset = 0;
      if (l >= 1) {
        const int pn = t.path[(size_t)(l - 1) * ps + li];
        pvp = t.stat[nidx(t, pn, i)].reward;
        reset = t.meta[nidx(t, pn, i)].is_reset;
      }
      float tr = s.reward - pvp;
      const float q = tr + disc * v;
      if (q > mm.x) mm.x = q;
      if (q < mm.y) mm.y = q;
      if (reset == 1) tr = s.reward;
      if (to_play == -1 || ntp != to_play)
        b = tr + disc * b;
      else
        b = -tr + disc * b;
    }
  }
  *mm_ptr = mm;
}

template <bool EZ>
__device__ inline void backup(const TreeView &t, int i, float4 *mm_ptr, int to_play, float value, float disc) {
  backup_slice<EZ>(t, i, i, t.B, mm_ptr, to_play, value, disc);
}

// expand_leaf with one lane per child (MuZero; all 64 lanes of the wave call it, A <= 64).
// Bit-identical: pmax is a max (order-free), the prior denominator is summed in action order by a
// readlane chain, every other quantity is per child.
// part: 0 = the whole expansion, 1 = the leaf's own record only (meta, reward), 2 = its children only
// (priors, fresh records): the two halves touch disjoint nodes, so two waves can run them at once.
__device__ inline void expand_wave(const TreeView &t, int i, int leaf, int to_play, int latent, float reward,
                                   const float *logits, int is_reset = -1, const uint64_t *exptab = kExp2fTab,
                                   int part = 0) {
  const int lane = threadIdx.x & 63;
  const int A = t.A;
  if (part != 2 && lane == 0) {
    NodeMeta m = t.meta[nidx(t, leaf, i)];
    m.latent = latent;
    m.to_play = to_play;
    if (is_reset >= 0) m.is_reset = is_reset;  // EfficientZero (is_reset < 0: MuZero, untouched)
    t.meta[nidx(t, leaf, i)] = m;
    t.stat[nidx(t, leaf, i)].reward = reward;
  }
  if (part == 1) return;
  const bool act = lane < A;
  const float lg = act ? logits[lane] : -INFINITY;
  const float pmax = fmaxf(kFloatMin, wave_max_dpp(lg));
  const float e = act ? glibc_expf(lg - pmax, exptab) : 0.0f;
  float sum = 0.0f;
  for (int a = 0; a < A; ++a) sum += readlane_f(e, a);
  if (act) {
    const int c = 1 + A * latent + lane;
    NodeStat cs;
    cs.visit = 0;
    cs.value_sum = 0.0f;
    cs.prior = e / sum;
    cs.reward = 0.0f;
    t.stat[nidx(t, c, i)] = cs;
    NodeMeta cm;
    cm.latent = -1;
    cm.to_play = 0;
    cm.best = -1;
    cm.is_reset = 0;
    t.meta[nidx(t, c, i)] = cm;
    if (t.val) t.val[nidx(t, c, i)] = 0.0f;
  }
}

// backup_slice<false> with one lane per path level (all 64 lanes call it). The bootstrap value is
// the only serial quantity: it runs leaf to root in registers (readlane chain, the reference's
// exact operation order), then every level updates its node, value cache and q in parallel; the
// min-max update is an order-free max / min (exact). Paths longer than 64 levels take several
// rounds. Also writes best_action along the path (cnode.cpp:806).
__device__ inline void backup_wave(const TreeView &t, int i, int li, int ps, float4 *mm_ptr, int to_play, float value,
                                   float disc) {
  const int lane = threadIdx.x & 63;
  const int len = t.pathlen[li];
  for (int l = lane; l < len; l += 64)
    t.meta[nidx(t, t.path[(size_t)l * ps + li], i)].best = t.path_act[(size_t)l * ps + li];
  float b = value;  // wave-uniform chain value
  float qmax = -INFINITY, qmin = INFINITY;
  for (int g0 = len; g0 >= 0; g0 -= 64) {
    const int l = g0 - lane;  // lane j holds level g0 - j (leaf-most first)
    const bool act = l >= 0;
    int node = 0, ntp = 0;
    NodeStat s;
    s.visit = 0; s.value_sum = 0.0f; s.prior = 0.0f; s.reward = 0.0f;
    if (act) {
      node = t.path[(size_t)l * ps + li];
      s = t.stat[nidx(t, node, i)];
      ntp = t.meta[nidx(t, node, i)].to_play;
    }
    const int nlev = g0 + 1 < 64 ? g0 + 1 : 64;
    float bl = 0.0f;
    for (int j = 0; j < nlev; ++j) {
      if (lane == j) bl = b;
      const float tr = readlane_f(s.reward, j);
      if (to_play == -1) {
        b = tr + disc * b;
      } else {
        const int nj = __builtin_amdgcn_readlane(ntp, j);
        b = (nj == to_play) ? (-tr + disc * b) : (tr + disc * b);
      }
    }
    if (act) {
      if (to_play == -1 || ntp == to_play)
        s.value_sum += bl;
      else
        s.value_sum += -bl;
      s.visit += 1;
      t.stat[nidx(t, node, i)] = s;
      const float v = node_value(s);
      if (t.val) t.val[nidx(t, node, i)] = v;
      const float q = (to_play == -1) ? s.reward + disc * v : s.reward + disc * -v;
      qmax = fmaxf(qmax, q);
      qmin = fminf(qmin, q);
    }
  }
  qmax = wave_max_dpp(qmax);
  qmin = -wave_max_dpp(-qmin);
  if (lane == 0) {
    float4 mm = *mm_ptr;
    if (qmax > mm.x) mm.x = qmax;
    if (qmin < mm.y) mm.y = qmin;
    *mm_ptr = mm;
  }
}

// backup_slice<true> with one lane per path level (EfficientZero cbackpropagate,
// ctree_efficientzero/lib/cnode.cpp:482-575). Per level: true_reward = value_prefix - parent's
// value_prefix feeds the min-max update, its is_reset form (the node's own value_prefix when the
// parent is reset) feeds the bootstrap chain. The chain runs leaf to root by readlane in the
// reference's order; the rest is per level; min-max by an order-free max / min (exact).
__device__ inline void backup_wave_ez(const TreeView &t, int i, int li, int ps, float4 *mm_ptr, int to_play,
                                      float value, float disc) {
  const int lane = threadIdx.x & 63;
  const int len = t.pathlen[li];
  float b = value;  // wave-uniform chain value
  float qmax = -INFINITY, qmin = INFINITY;
  for (int g0 = len; g0 >= 0; g0 -= 64) {
    const int l = g0 - lane;  // lane j holds level g0 - j (leaf-most first)
    const bool act = l >= 0;
    int node = 0, ntp = 0;
    NodeStat s;
    s.visit = 0; s.value_sum = 0.0f; s.prior = 0.0f; s.reward = 0.0f;
    float tq = 0.0f, tc = 0.0f;  // true reward for the min-max update / for the chain
    if (act) {
      node = t.path[(size_t)l * ps + li];
      s = t.stat[nidx(t, node, i)];
      ntp = t.meta[nidx(t, node, i)].to_play;
      float pvp = 0.0f;
      int reset = 0;
      if (l >= 1) {
        const int pn = t.path[(size_t)(l - 1) * ps + li];
        pvp = t.stat[nidx(t, pn, i)].reward;
        reset = t.meta[nidx(t, pn, i)].is_reset;
      }
      tq = s.reward - pvp;
      tc = (reset == 1) ? s.reward : tq;
    }
    const int nlev = g0 + 1 < 64 ? g0 + 1 : 64;
    float bl = 0.0f;
    for (int j = 0; j < nlev; ++j) {
      if (lane == j) bl = b;
      const float tr = readlane_f(tc, j);
      if (to_play == -1) {
        b = tr + disc * b;
      } else {
        const int nj = __builtin_amdgcn_readlane(ntp, j);
        b = (nj != to_play) ? (tr + disc * b) : (-tr + disc * b);
      }
    }
    if (act) {
      if (to_play == -1 || ntp == to_play)
        s.value_sum += bl;
      else
        s.value_sum += -bl;
      s.visit += 1;
      t.stat[nidx(t, node, i)] = s;
      const float v = node_value(s);
      if (t.val) t.val[nidx(t, node, i)] = v;
      const float q = tq + disc * v;
      qmax = fmaxf(qmax, q);
      qmin = fminf(qmin, q);
    }
  }
  qmax = wave_max_dpp(qmax);
  qmin = -wave_max_dpp(-qmin);
  if (lane == 0) {
    float4 mm = *mm_ptr;
    if (qmax > mm.x) mm.x = qmax;
    if (qmin < mm.y) mm.y = qmin;
    *mm_ptr = mm;
  }
}

// h^-1 of InverseScalarTransform (scaling_transform.py:123-127), eps = 0.001.
__device__ inline float h_inverse(float value) {
  const float eps = 0.001f;
  float tmp = (sqrtf(1.0f + 0.004f * (fabsf(value) + 1.0f + eps)) - 1.0f) * (1.0f / 0.002f);
  float sgn = value > 0.0f ? 1.0f : (value < 0.0f ? -1.0f : 0.0f);
  return sgn * (tmp * tmp - 1.0f);
}

// CRoots::prepare / prepare_no_noise (cnode.cpp:321-358): expand each root over its legal list
// (an empty list means every action, cnode.cpp:101-107), optional Dirichlet mix
// (add_exploration_noise :149-167), visit_count = 1.
struct PrepareArgs {
  NodeStat *stat;
  NodeMeta *meta;
  int32_t *legal, *nlegal;
  const int32_t *legal_in, *count_in, *to_play;
  const float *noises, *rewards, *logits;
  float noise_weight;
  int B, A;
};

// lg: the root's policy logits (null: p.logits row i; lzm_conv_heads_prepare passes its LDS copy)
__device__ inline void prepare_root(const PrepareArgs &p, int i, const float *lg = nullptr) {
  const int A = p.A;
  int n = p.count_in[i];
  if (n <= 0) {
    n = A;
    for (int a = 0; a < A; ++a) p.legal[(size_t)i * A + a] = a;
  } else {
    for (int j = 0; j < A; ++j) p.legal[(size_t)i * A + j] = j < n ? p.legal_in[(size_t)i * A + j] : -1;
  }
  p.nlegal[i] = n;
  if (!lg) lg = p.logits + (size_t)i * A;
  float pmax = kFloatMin;
  for (int j = 0; j < n; ++j) {
    const float l = lg[p.legal[(size_t)i * A + j]];
    if (pmax < l) pmax = l;
  }
  float sum = 0.0f;
  for (int j = 0; j < n; ++j) sum += glibc_expf(lg[p.legal[(size_t)i * A + j]] - pmax);
  const float f = p.noise_weight;
  for (int j = 0; j < n; ++j) {
    const int a = p.legal[(size_t)i * A + j];
    float prior = glibc_expf(lg[a] - pmax) / sum;
    if (p.noises) {
      const float noise = p.noises[(size_t)i * A + j];
      prior = prior * (1 - f) + noise * f;
    }
    NodeStat c;
    c.visit = 0;
    c.value_sum = 0.0f;
    c.prior = prior;
    c.reward = 0.0f;
    p.stat[(size_t)(1 + a) * p.B + i] = c;
    NodeMeta cm;
    cm.latent = -1;
    cm.to_play = 0;
    cm.best = -1;
    cm.is_reset = 0;
    p.meta[(size_t)(1 + a) * p.B + i] = cm;
  }
  NodeStat r;
  r.visit = 1;
  r.value_sum = 0.0f;
  r.prior = 0.0f;
  r.reward = p.rewards[i];
  p.stat[i] = r;
  NodeMeta rm;
  rm.latent = 0;
  rm.to_play = p.to_play[i];
  rm.best = -1;
  rm.is_reset = 0;
  p.meta[i] = rm;
}

}  // namespace lzm
