// lzm_search_res.h — the fused MuZero search with the network resident on the CU (CartPole shape).
//
// Same contract as search_mlp_kernel (lzm_search_mlp.h: one launch = every simulation of a
// MuZeroMCTSCtree.search, mcts_ctree.py:255-321), specialised to the MuZeroModelMLP shape of
// BASELINE.json config 2 — latent 128, head hidden 32, reward/value supports 601,
// res_connection_in_dynamics (muzero_model_mlp.py:179-204, :327-440; common.py:883-971) — with one
// root per workgroup. What changes is where the 149 K weights live. search_mlp_kernel streams all
// of them from L2 every simulation (≈0.6 MiB per CU per simulation, which its phase stamps show
// as the largest cost). Here a 256-thread workgroup (one wave per SIMD, so up to ≈450 registers
// per lane) keeps them on the CU for the whole launch:
//   registers: fc_dynamics_2[1], fc_prediction_common[0..1], the reward / value / policy head
//              hiddens and the policy output                                  (≈245 floats/lane)
//   LDS:       fc_dynamics[1], fc_dynamics_2[0]                                (2 x 64 KiB)
//   streamed:  fc_dynamics[0] (latent rows) and the two 32 -> 601 support heads, ≈0.2 MiB per
//              simulation, each prefetched into one 80-register buffer several steps (or, for
//              the first layer, a whole tree phase) ahead of its use.
// Every 128 x 128 layer uses one lane mapping: lane l computes column l >> 1 over K half l & 1 and
// the halves meet by one DPP swap. The one-hot action rows of fc_dynamics[0] are never multiplied:
// the action's row is added after the latent rows (the exact value of the one-hot product), so the
// layer can start before the action is known.
//
// Tree phase (R = 1): wave 0 walks the tree (descend_wave, bit-exact with the reference). In
// parity mode the reference's single rand() stream makes root i's draws start at the sum of the
// depths of roots < i; every workgroup publishes its depth at once (lzm_search_mlp.h, decoupled
// look-back), but only a root whose walk stopped at a tie among unexpanded children needs the
// draw VALUE — and that tie leaves the leaf's parent (the gathered latent) known, only the action
// open. So the look-back wait is deferred behind the first layer's latent rows and skipped
// entirely when no draw value is needed. A tie reaching an expanded child (depth depends on the
// draw) is resolved serially before the gather, as in search_mlp_kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_search_mlp.h"
#include "lzm_tree.h"

namespace lzm {

constexpr int kRT = 256;  // threads: one wave per SIMD
constexpr int kRWaves = kRT / 64;
constexpr int kRHid = 128, kRF = 32, kRV = 601;
constexpr int kRMaxA = 32;                 // policy output: 8 lanes per action
constexpr int kRTail = kRV - 2 * kRT;      // support columns past two full lane rounds (89)
static_assert(kRTail > 0 && 2 * kRTail <= kRT, "support tail: two lanes per column");
// float4 slots (each kRT lanes wide) per resident block
constexpr int kRSlotsD = 16, kRSlotsRH = 4, kRSlotsVPH = 8, kRSlotsS = 20, kRSlotsPO = 1;

// D-block lane map (every 128 x 128 layer). LZM_RES_D4 = 1 (default): lane l owns the four columns
// 4 (l >> 3) .. +3 over the K eighth 16 (l & 7) .. +15, so it reads 4 activation float4 per row (all in
// flight at once) and uses each for 4 columns; the 8 lanes of a column group meet by a 3-step DPP
// butterfly that leaves column 4 (l >> 3) + ((l & 7) >> 1) in lane pair (l, l ^ 1) (reduce_d4). 0: lane
// l owns column l >> 1 over K half l & 1 (16 activation float4 per row, read through a shallow
// software pipeline for lack of registers). Same weights per lane either way.
#ifndef LZM_RES_D4
#define LZM_RES_D4 1
#endif
// LZM_RES_EGATHER (default 1): the walking wave gathers the leaf's parent latent X0 itself, right
// after its walk when x is final (the walk's barrier orders it), or after a status-2 root's draw
// resolution: the gather phase's own barrier and its dependent load after it go.
#ifndef LZM_RES_EGATHER
#define LZM_RES_EGATHER 1
#endif
// LZM_RES_SEEDW1 (default 1): this simulation's glibc seed state (s_z0, read only after the walk) is
// computed by wave 1 during wave 0's walk instead of by wave 0 before the terms pass's barrier:
// +0.8% with random and with zero-init heads (profiles/r04/ab_rd5e_seedw1.txt).
#ifndef LZM_RES_SEEDW1
#define LZM_RES_SEEDW1 1
#endif
// Measured and removed in round 4 (DESIGN.md §9 gives each A/B): wave 0 computing the pUCT terms
// alone with an early latent gather, wave 0's fc_dynamics[0] prefetch in quarters, a two-column
// value / policy head hidden layer, a one-barrier support softmax, the late draw from a window of
// draws built during the walk, fc_prediction_common[1] prefetched during the look-back.
constexpr int kDwinBack = 20;  // draw window [base_prev - kDwinBack, base_prev - kDwinBack + 64)
// LZM_RES_DWIN2 (default 1, parity mode, A = 2): a tie between visited children (status 2/3: the
// walk's remaining levels need draws, the zero-init-heads regime at nearly every simulation) waits
// for its look-back with wave 0 alone (lookback_sum_w0) while wave 1 computes the window of draws
// around the previous look-back base, so the resumed walk reads its draws from LDS instead of a
// coefficient-row round trip per lane after the wait (positions outside the window: the rows).
#ifndef LZM_RES_DWIN2
#define LZM_RES_DWIN2 1
#endif
// LZM_RES_SPEC_PATH (default 1): a status-3 root (depth speculated over all draw patterns) resolves
// its path after the look-back from the matching pattern lane's choice bits (speculate_depth_a2) —
// a pointer chase — instead of re-walking the tie subtree with scores.
#ifndef LZM_RES_SPEC_PATH
#define LZM_RES_SPEC_PATH 1
#endif

// Part `part` (0..2: coefficient words 11 part .. 11 part + 10) of the window's 64 dot products, added
// to win (the sums are mod 2^32, so the three waves' LDS adds may land in any order); win must be zero
// before the first add and holds (sum) before the >> 1 of the draw. Eleven loads per lane.
__device__ __forceinline__ void dwin_add_part(const uint32_t *coef, int npos, const uint32_t *z0, int lo, uint32_t *win,
                                              int part) {
  const int lane = threadIdx.x & 63;
  const int q = lo + lane;
  const int j0 = 11 * part, j1 = part == 2 ? 31 : j0 + 11;
  if (q < npos) {
    const uint32_t *c = coef + (size_t)q * 31;
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 11; ++j)
      if (j0 + j < j1) v += c[j0 + j] * z0[j0 + j];
    __hip_atomic_fetch_add(win + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// The draw of this lane's level lo + lane of a resumed walk from the window win[0..64) of stream
// positions dlo..; *miss when a level below hi lies outside it.
__device__ __forceinline__ uint32_t window_draw(int npos, int base, int lo, int hi, const uint32_t *win, int dlo,
                                                bool *miss) {
  const int lane = threadIdx.x & 63;
  const int q = base + lo + lane, o = q - dlo;
  *miss = false;
  if (lo + lane >= hi || q >= npos) return 0u;
  if (o >= 0 && o < 64) return win[o] >> 1;
  *miss = true;
  return 0u;
}

// Resident weight layout (lzm_mlp_prepare writes it after the generic kernel layout; res_source
// below is its definition). Every block is [slot][lane] float4, so a wave-instruction of a block
// is one contiguous 1 KiB read.
//   D (128 x 128, six of them): slot j, lane l: W[16 (l & 7) + 4 (j >> 2) .. +3][4 (l >> 3) + (j & 3)]
//      (LZM_RES_D4; else W[64 (l & 1) + 4 j .. +3][l >> 1])
//   RH (128 -> 32 reward head hidden): slot j < 4: W[16 (l & 7) + 4 j ..][l >> 3]
//   VPH (128 -> 64: [value hidden | policy hidden]): slot j < 8: W[32 (l & 3) + 4 j ..][l >> 2]
//   S (32 -> 601 support head): slots 0-7: column l, k = 4 j; slots 8-15: column 256 + l;
//      slots 16-19: column 512 + (l >> 1), k = 16 (l & 1) + 4 (j - 16), lanes < 2 * kRTail
//   PO (32 -> A policy output): one slot: W[4 (l & 7) ..][l >> 3], l >> 3 < A
// then the biases ([6][128] D, [32] RH, [64] VPH, [604] RS, [604] VS, [32] PO) and the one-hot
// action rows of fc_dynamics[0], [A][128].
// dynamic LDS plan of the resident kernel (float offsets; res_plan below)
struct ResPlan {
  int wd1, wd2, stat, meta, lut, legal, val, path, pact, act, l2n, nq, cs, dec, misc, pbt, pbt_rows, floats;
};
struct ResNet {
  // the resident layout (one base pointer: every block offset but the action rows' is a
  // compile-time constant, res_block_offset; the kernel derives the block addresses, which keeps
  // ~30 scalar registers of block pointers out of the simulation loop)
  const float *w;
  // LDS float offsets beyond SearchArgs' tree plan
  ResPlan plan;      // dynamic LDS plan (res_plan)
  int select_mode;  // LZM_RES_SELECT (experiments): how the walk runs, see the simulation loop
  int late_draw;    // NR = 1: two-way leaf ties run the dynamics layers for both candidates before the
                    // look-back wait (LZM_RES_LATE, default 1)
  int spec_depth;   // status-2 ties: publish the depth early when every draw outcome gives the same
                    // depth (speculate_depth_a2; LZM_RES_SPEC_DEPTH, default 1)
};

// floats of the bias blocks ([6][128] D, [32] RH, [64] VPH, [604] RS, [604] VS, [32] PO)
constexpr int kResBiasFloats = 6 * 128 + 32 + 64 + 2 * 604 + 32;
enum ResBlock { kRbD = 0, kRbRH = 6, kRbVPH, kRbRS, kRbVS, kRbPO, kRbBD, kRbBRH, kRbBVPH, kRbBRS, kRbBVS, kRbBPO, kRbAct, kRbN };

// float count of each block (A actions)
__host__ __device__ inline size_t res_block_floats(int b, int A) {
  if (b < kRbRH) return (size_t)kRSlotsD * kRT * 4;
  switch (b) {
    case kRbRH: return (size_t)kRSlotsRH * kRT * 4;
    case kRbVPH: return (size_t)kRSlotsVPH * kRT * 4;
    case kRbRS: case kRbVS: return (size_t)kRSlotsS * kRT * 4;
    case kRbPO: return (size_t)kRSlotsPO * kRT * 4;
    case kRbBD: return 6 * kRHid;
    case kRbBRH: return kRF;
    case kRbBVPH: return 2 * kRF;
    case kRbBRS: case kRbBVS: return (kRV + 3) & ~3;
    case kRbBPO: return kRMaxA;
    default: return (size_t)A * kRHid;
  }
}
__host__ __device__ inline size_t res_block_offset(int b, int A) {
  size_t o = 0;
  for (int q = 0; q < b; ++q) o += res_block_floats(q, A);
  return o;
}

// block b of the resident layout (b < kRbAct: a compile-time offset)
__device__ __forceinline__ const float4 *res_blk4(const ResNet &n, int b) {
  return reinterpret_cast<const float4 *>(n.w + res_block_offset(b, 0));
}
__device__ __forceinline__ const float *res_blk(const ResNet &n, int b, int A) { return n.w + res_block_offset(b, A); }

// Packed-network source of resident float d of block b: packed layer index (lzm_kernels.hip
// mlp_shapes order: 0,1 fc_dynamics, 2,3 fc_dynamics_2, 4,5 reward head, 6,7 prediction common,
// 8,9 value head, 10,11 policy head), row k (k < 0: the bias) and column; layer < 0: zero padding.
__host__ __device__ inline void res_source(int b, size_t d, int A, int *layer, int *k, int *col) {
  *layer = -1; *k = 0; *col = 0;
  const int e = (int)(d & 3);
  const int f4 = (int)(d >> 2);
  const int j = f4 / kRT, l = f4 % kRT;
  if (b < kRbRH) {
    const int src[6] = {0, 1, 2, 3, 6, 7};
    *layer = src[b];
#if LZM_RES_D4
    *col = 4 * (l >> 3) + (j & 3); *k = 16 * (l & 7) + 4 * (j >> 2) + e;
#else
    *col = l >> 1; *k = 64 * (l & 1) + 4 * j + e;
#endif
    return;
  }
  switch (b) {
    case kRbRH: *layer = 4; *col = l >> 3; *k = 16 * (l & 7) + 4 * j + e; return;
    case kRbVPH: {
      const int c = l >> 2;
      *layer = c < kRF ? 8 : 10; *col = c < kRF ? c : c - kRF; *k = 32 * (l & 3) + 4 * j + e;
      return;
    }
    case kRbRS: case kRbVS: {
      const int ly = b == kRbRS ? 5 : 9;
      if (j < 8) { *layer = ly; *col = l; *k = 4 * j + e; }
      else if (j < 16) { *layer = ly; *col = kRT + l; *k = 4 * (j - 8) + e; }
      else if (l < 2 * kRTail) { *layer = ly; *col = 2 * kRT + (l >> 1); *k = 16 * (l & 1) + 4 * (j - 16) + e; }
      return;
    }
    case kRbPO: if ((l >> 3) < A) { *layer = 11; *col = l >> 3; *k = 4 * (l & 7) + e; } return;
    case kRbBD: {
      const int src[6] = {0, 1, 2, 3, 6, 7};
      *layer = src[d / kRHid]; *k = -1; *col = (int)(d % kRHid);
      return;
    }
    case kRbBRH: *layer = 4; *k = -1; *col = (int)d; return;
    case kRbBVPH: *layer = d < (size_t)kRF ? 8 : 10; *k = -1; *col = (int)(d % kRF); return;
    case kRbBRS: case kRbBVS: if (d < (size_t)kRV) { *layer = b == kRbBRS ? 5 : 9; *k = -1; *col = (int)d; } return;
    case kRbBPO: if (d < (size_t)A) { *layer = 11; *k = -1; *col = (int)d; } return;
    default: *layer = 0; *k = kRHid + (int)(d / kRHid); *col = (int)(d % kRHid); return;
  }
}

// NS float4 slots of a resident block into registers (buffer loads: the slot offset is scalar)
template <int NS, int J0 = 0, int J1 = NS>
__device__ __forceinline__ void res_fetch(const float4 *blk, float4 *dst) {
  const __amdgpu_buffer_rsrc_t r = wave_rsrc(blk, NS * kRT * 16);
  const int vo = (int)threadIdx.x * 16;
#pragma unroll
  for (int j = J0; j < J1; ++j) {
    const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, j * kRT * 16, 0);
    dst[j] = make_float4(v.x, v.y, v.z, v.w);
  }
}

// Partial dot product of 4*NJ consecutive inputs x4[0..NJ) with weights w(j): four independent
// FMA chains (k mod 4), summed as (c0 + c1) + (c2 + c3).
// (LZM_PK_FMA: the chains in pairs, v_pk_fma_f32 — each half rounds exactly like v_fma_f32)
#ifndef LZM_PK_FMA
#define LZM_PK_FMA 1
#endif
typedef float lzm_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void fma4(float4 v, float4 q, float *a) {
#if LZM_PK_FMA
  lzm_f2 lo = {a[0], a[1]}, hi = {a[2], a[3]};
  lo = __builtin_elementwise_fma((lzm_f2){v.x, v.y}, (lzm_f2){q.x, q.y}, lo);
  hi = __builtin_elementwise_fma((lzm_f2){v.z, v.w}, (lzm_f2){q.z, q.w}, hi);
  a[0] = lo.x; a[1] = lo.y; a[2] = hi.x; a[3] = hi.y;
#else
  a[0] = __fmaf_rn(v.x, q.x, a[0]);
  a[1] = __fmaf_rn(v.y, q.y, a[1]);
  a[2] = __fmaf_rn(v.z, q.z, a[2]);
  a[3] = __fmaf_rn(v.w, q.w, a[3]);
#endif
}
template <int NJ, typename WF>
__device__ __forceinline__ float dot4(const float4 *x4, WF w) {
  float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int j = 0; j < NJ; ++j) fma4(x4[j], w(j), a);
  return (a[0] + a[1]) + (a[2] + a[3]);
}

// 128-wide activation rows in LDS are padded: the upper 64 floats start 4 floats after the lower
// ones (row stride kRRow), so the two lanes of a pair, which read float4 j of their half, hit
// different banks (unpadded, the halves are 256 B apart: the same bank, a 2-way conflict on every
// activation read of every dense layer). rpad(c): column c's float offset in a padded row.
constexpr int kRRow = kRHid + 4;
constexpr int kRHalf4 = kRHid / 8 + 1;  // float4 offset of the upper half
__device__ __forceinline__ int rpad(int c) { return c + ((c >> 6) << 2); }

// The column of a 128 x 128 layer this lane's result holds (both lanes of the pair (l, l ^ 1) hold
// it; the even lane writes it).
__device__ __forceinline__ int d_col() {
#if LZM_RES_D4
  return 4 * ((int)threadIdx.x >> 3) + (((int)threadIdx.x & 7) >> 1);
#else
  return (int)threadIdx.x >> 1;
#endif
}

// LZM_RES_D4: the four column partials h0..h3 of the 8 lanes of a column group to full sums —
// lanes e and 7 - e (row_half_mirror) split the columns {0, 1} / {2, 3}, lanes e and e ^ 2 split the
// pair, lanes e and e ^ 1 add: column (e >> 1) ends in lanes e, e ^ 1 (the same bits in both: the last
// add is commutative). A fixed order, so every launch rounds the same way.
__device__ __forceinline__ float reduce_d4(float h0, float h1, float h2, float h3) {
  const int e = threadIdx.x & 7;
  const bool lo = e < 4;
  float k0 = lo ? h0 : h2, k1 = lo ? h1 : h3;
  const float s0 = lo ? h2 : h0, s1 = lo ? h3 : h1;
  k0 += dpp_f<0x141>(s0);
  k1 += dpp_f<0x141>(s1);
  const bool q = (e & 2) == 0;
  float m = q ? k0 : k1;
  const float snd = q ? k1 : k0;
  m += dpp_f<0x4E>(snd);
  return m + dpp_f<0xB1>(m);
}

// Full pre-activation of this lane's column (d_col) of a 128 x 128 layer.
template <typename WF>
__device__ __forceinline__ float dense128(const float *x, WF w) {
#if LZM_RES_D4
  const int e = threadIdx.x & 7;
  const float4 *x4 = reinterpret_cast<const float4 *>(x) + 4 * e + (e >> 2);
  float4 xv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) xv[j] = x4[j];
  float a[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) a[c][0] = a[c][1] = a[c][2] = a[c][3] = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) fma4(xv[j], w(4 * j + c), a[c]);
  return reduce_d4((a[0][0] + a[0][1]) + (a[0][2] + a[0][3]), (a[1][0] + a[1][1]) + (a[1][2] + a[1][3]),
                   (a[2][0] + a[2][1]) + (a[2][2] + a[2][3]), (a[3][0] + a[3][1]) + (a[3][2] + a[3][3]));
#else
  const float h = dot4<16>(reinterpret_cast<const float4 *>(x) + kRHalf4 * (threadIdx.x & 1), w);
  return h + dpp_f<0xB1>(h);
#endif
}

// Logits of one support head (input: 32 floats in LDS; weights: the 20-slot buffer P): lane l
// gets columns l, 256 + l and (l < 2 * kRTail, l even) 512 + (l >> 1).
__device__ __forceinline__ void support_logits(const float *h, const float4 *P, const float *bias, float &z0, float &z1,
                                               float &z2) {
  const int tid = threadIdx.x;
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  z0 = dot4<8>(h4, [&](int j) { return P[j]; }) + bias[tid];
  z1 = dot4<8>(h4, [&](int j) { return P[8 + j]; }) + bias[kRT + tid];
  const float t = dot4<4>(h4 + 4 * (tid & 1), [&](int j) { return P[16 + j]; });
  z2 = (t + dpp_f<0xB1>(t)) + (tid < 2 * kRTail ? bias[2 * kRT + (tid >> 1)] : 0.0f);
}

// Two-action selection outcome of an expanded node when it does not depend on the walk (all
// children visited, or a single legal child): 0 / 1 = the legal position cselect_child picks,
// 3 = a tie between the two visited children (a draw decides), 2 = depends on the walk's mean-q
// (an unvisited child scores the normalised parent mean-q). Same operations as the walk's scores.
__device__ __forceinline__ int a2_decision(float4 c0, float4 c1, int n) {
  if (n < 2) return 0;
  if (!__float_as_int(c0.w) || !__float_as_int(c1.w)) return 2;
  const float s0 = c0.x + c0.y, s1 = c1.x + c1.y;
  const float M = fmaxf(s0, s1);
  const int r = (s0 == M) ? 0 : 1;
  return (r == 0 && s1 >= M - 0.000001f) ? 3 : r;
}

// ---- selection split in two (MuZero, tree slice in LDS, one root):
// (1) every expanded node's pUCT terms that do not depend on the walk, one thread per node
//     (cucb_score, cnode.cpp:655-699: prior_score, and for visited children the normalised,
//     clamped value term; compute_mean_q's sums over visited children, cnode.cpp:169-203);
// (2) the walk itself (wave 0), left with the mean-q chain (the only walk-dependent term: it is
//     what unvisited children score) and the argmax / tie list per level.
// Same float operations in the same order as descend_wave, so the same bits.
// nq[latent] = {total_q, total_v}; cs[child node] = {prior_score, value term, child latent, visited}
// dec (nullable, A == 2): each node's walk-independent outcome (a2_decision) for descend_a2.
// node_terms: one expanded node n (latent L), by the calling thread.
__device__ inline void node_terms(const TreeView &t, int L, int n, float2 *nq, float4 *cs, float4 mm, int players,
                                  float disc, int *dec) {
  {
    const NodeStat s = t.stat[n];
    const int nleg = legal_n(t, 0, n);
    const int base = 1 + t.A * L;
    int N = s.visit - 1;
    N = N < 0 ? 0 : (N >= t.lut_n ? t.lut_n - 1 : N);
    const float2 Lx = t.lut[N];
    float total_q = 0.0f;
    int total_v = 0;
    float4 c01[2];
    for (int j = 0; j < nleg; ++j) {
      const int c = base + legal_at(t, 0, n, j);
      const NodeStat cst = t.stat[c];
      const float cv = t.val[c];
      const float tr = cst.reward;
      float vv = 0.0f;
      if (cst.visit > 0) {
        total_q += tr + disc * cv;
        ++total_v;
        float v = (players == 1) ? tr + disc * cv : tr + disc * (-cv);
        v = mm_normalize(mm, v);
        if (v < 0) v = 0;
        if (v > 1) v = 1;
        vv = v;
      }
      float pb_c = Lx.x;
      pb_c *= (t.pbt && cst.visit <= N) ? t.pbt[N * (N + 1) / 2 + cst.visit] : (Lx.y / (float)(cst.visit + 1));
      const float4 term = make_float4(pb_c * cst.prior, vv, __int_as_float(t.meta[c].latent),
                                      __int_as_float(cst.visit > 0 ? 1 : 0));
      cs[c] = term;
      if (j < 2) c01[j] = term;
    }
    nq[L] = make_float2(total_q, __int_as_float(total_v));
    if (dec) dec[L] = (t.A == 2 && nleg >= 1) ? a2_decision(c01[0], c01[nleg > 1 ? 1 : 0], nleg) : 2;
  }
}
__device__ inline void precompute_terms(const TreeView &t, int nlat, const int *lat2node, float2 *nq, float4 *cs,
                                        float4 mm, int players, float disc, int *dec = nullptr) {
  for (int L = threadIdx.x; L < nlat; L += kRT) {
    const int n = lat2node[L];
    if (n >= 0) node_terms(t, L, n, nq, cs, mm, players, disc, dec);
  }
}

// node_terms for two actions, written for few LDS round trips: a child's slot depends on the latent
// only (1 + 2 L + legal position; the root, latent 0, takes its legal actions from registers), so
// both children's records are read with the latent -> node map, the node's visit count next, then
// the pb_c table row; every read is unconditional and the branches are selects. Same float
// operations in the same order as node_terms (so the same bits), and also dec[L].
__device__ inline void precompute_terms_a2(const TreeView &t, int nlat, const int *lat2node, float2 *nq, float4 *cs,
                                           float4 mm, int players, float disc, int *dec, const int *rleg,
                                           int nleg_root) {
  for (int L = threadIdx.x; L < nlat; L += kRT) {
    const int n = lat2node[L];
    const bool root = L == 0;
    const int nleg = root ? nleg_root : 2;
    const int base = 1 + 2 * L;
    const int c0 = base + (root ? rleg[0] : 0);
    const int c1 = base + (root ? rleg[nleg > 1 ? 1 : 0] : 1);
    const NodeStat s0 = t.stat[c0], s1 = t.stat[c1];
    const float v0 = t.val[c0], v1 = t.val[c1];
    const int l0 = t.meta[c0].latent, l1 = t.meta[c1].latent;
    if (n < 0) continue;
    int N = t.stat[n].visit - 1;
    N = N < 0 ? 0 : (N >= t.lut_n ? t.lut_n - 1 : N);
    const float2 Lx = t.lut[N];
    const int row = N * (N + 1) / 2;
    const bool p0 = t.pbt && s0.visit <= N, p1 = t.pbt && s1.visit <= N;
    const float f0 = p0 ? t.pbt[row + s0.visit] : (Lx.y / (float)(s0.visit + 1));
    const float f1 = p1 ? t.pbt[row + s1.visit] : (Lx.y / (float)(s1.visit + 1));
    float total_q = 0.0f;
    int total_v = 0;
    float vv0 = 0.0f, vv1 = 0.0f;
    if (s0.visit > 0) {
      total_q += s0.reward + disc * v0;
      ++total_v;
      float v = (players == 1) ? s0.reward + disc * v0 : s0.reward + disc * (-v0);
      v = mm_normalize(mm, v);
      if (v < 0) v = 0;
      if (v > 1) v = 1;
      vv0 = v;
    }
    if (nleg > 1 && s1.visit > 0) {
      total_q += s1.reward + disc * v1;
      ++total_v;
      float v = (players == 1) ? s1.reward + disc * v1 : s1.reward + disc * (-v1);
      v = mm_normalize(mm, v);
      if (v < 0) v = 0;
      if (v > 1) v = 1;
      vv1 = v;
    }
    float pb0 = Lx.x, pb1 = Lx.x;
    pb0 *= f0;
    pb1 *= f1;
    const float4 t0 = make_float4(pb0 * s0.prior, vv0, __int_as_float(l0), __int_as_float(s0.visit > 0 ? 1 : 0));
    const float4 t1 = make_float4(pb1 * s1.prior, vv1, __int_as_float(l1), __int_as_float(s1.visit > 0 ? 1 : 0));
    if (nleg > 0) cs[c0] = t0;
    if (nleg > 1) cs[c1] = t1;
    nq[L] = make_float2(total_q, __int_as_float(total_v));
    dec[L] = nleg >= 1 ? a2_decision(t0, nleg > 1 ? t1 : t0, nleg) : 2;
  }
}

// The walk over the precomputed terms (descend_wave's contract and outputs; wave 0).
// Where a walk stands at the top of a level (a classification walk stops at a tie with the
// state of that level, so the resolution resumes there instead of walking from the root).
struct WalkState {
  int node, lat, len, plat, last_action, is_root, vtp;
  float parent_q;
};
__device__ inline WalkState walk_start(const TreeView &t, int vtp) {
  WalkState w;
  w.node = 0; w.lat = t.meta[0].latent; w.len = 0; w.plat = -1; w.last_action = -1; w.is_root = 1; w.vtp = vtp;
  w.parent_q = 0.0f;
  return w;
}

template <bool CLASSIFY, typename Draw>
__device__ inline Descent descend_terms(const TreeView &t, const float2 *nq, const float4 *cs, float4 mm, int vtp,
                                        int players, Draw draw, TieInfo *tie, WalkState *resume = nullptr,
                                        WalkState *at_tie = nullptr) {
  const int lane = threadIdx.x & 63;
  WalkState w0 = resume ? *resume : walk_start(t, vtp);
  int node = w0.node, is_root = w0.is_root, len = w0.len, last_action = w0.last_action, plat = w0.plat;
  float parent_q = w0.parent_q;
  int lat = w0.lat;
  vtp = w0.vtp;
  if (lane == 0 && !resume) t.path[0] = 0;
  if (CLASSIFY) tie->status = 0;
  while (lat >= 0 && len < t.depth_cap - 1) {
    if (CLASSIFY && at_tie) {
      at_tie->node = node; at_tie->lat = lat; at_tie->len = len; at_tie->plat = plat;
      at_tie->last_action = last_action; at_tie->is_root = is_root; at_tie->vtp = vtp; at_tie->parent_q = parent_q;
    }
    const int n = legal_n(t, 0, node);
    const int base = 1 + t.A * lat;
    const bool valid = lane < n;
    const int a = valid ? legal_at(t, 0, node, lane) : 0;
    const float4 c = valid ? cs[base + a] : make_float4(0.0f, 0.0f, __int_as_float(-1), __int_as_float(0));
    const float2 q = nq[lat];
    const int total_v = __float_as_int(q.y);
    float mean_q;
    if (is_root && total_v > 0)
      mean_q = q.x / (float)total_v;
    else
      mean_q = (parent_q + q.x) / (float)(total_v + 1);
    is_root = 0;
    parent_q = mean_q;
    float vu = mm_normalize(mm, mean_q);
    if (vu < 0) vu = 0;
    if (vu > 1) vu = 1;
    const float score = c.x + (__float_as_int(c.w) ? c.y : vu);
    const float M = wave_max_dpp(valid ? score : -INFINITY);
    const int r = __ffsll((long long)__ballot(valid && score == M)) - 1;
    const uint64_t mask = __ballot(valid && lane > r && score >= M - 0.000001f) | (1ull << r);
    const int nl = __popcll(mask);
    if (CLASSIFY && nl > 1) {
      const bool leaf_child = !((mask >> lane) & 1ull) || __float_as_int(c.z) < 0;
      const bool all_leaves = __ballot(!leaf_child) == 0ull;
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = mask;
      Descent d;
      d.len = len + 1;
      d.x = lat;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    const uint32_t rr = CLASSIFY ? 0u : draw(len);
    int kk = (int)(rr % (uint32_t)nl);
    uint64_t mm_ = mask;
    for (; kk > 0; --kk) mm_ &= mm_ - 1;
    const int jsel = __ffsll((long long)mm_) - 1;
    const int action = __builtin_amdgcn_readlane(a, jsel);
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    node = base + action;
    last_action = action;
    if (lane == 0) {
      t.path_act[len] = action;
      t.path[len + 1] = node;
    }
    ++len;
    plat = lat;
    lat = __builtin_amdgcn_readlane(__float_as_int(c.z), jsel);
  }
  Descent d;
  d.len = len;
  d.x = plat;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

// descend_terms for small action spaces (A <= AM <= 4): every lane of the wave evaluates the level
// (all AM children's terms as broadcast LDS reads, the max / first index / tie list as a short
// unrolled chain of per-lane compares), so a level is one round of LDS reads and a few dozen
// dependent VALU operations — no DPP reduction, ballots or readlanes on the chain. The root's legal
// actions (rleg, nleg) are passed in registers. Same float operations and tie rule as descend_terms
// (SURVEY.md A7 closed form), so the same bits; every lane returns the same Descent.
template <int AM, bool CLASSIFY, typename Draw>
__device__ inline Descent descend_small(const TreeView &t, const float2 *nq, const float4 *cs, float4 mm, int vtp,
                                        int players, const int *rleg, int nleg, Draw draw, TieInfo *tie,
                                        WalkState *resume = nullptr, WalkState *at_tie = nullptr) {
  const int lane = threadIdx.x & 63;
  const int A = t.A;
  WalkState w0 = resume ? *resume : walk_start(t, vtp);
  int node = w0.node, is_root = w0.is_root, len = w0.len, last_action = w0.last_action, plat = w0.plat;
  float parent_q = w0.parent_q;
  int lat = w0.lat;
  vtp = w0.vtp;
  if (lane == 0 && !resume) t.path[0] = 0;
  if (CLASSIFY) tie->status = 0;
  while (lat >= 0 && len < t.depth_cap - 1) {
    if (CLASSIFY && at_tie) {
      at_tie->node = node; at_tie->lat = lat; at_tie->len = len; at_tie->plat = plat;
      at_tie->last_action = last_action; at_tie->is_root = is_root; at_tie->vtp = vtp; at_tie->parent_q = parent_q;
    }
    const bool root = node == 0;
    const int n = root ? nleg : A;
    const int base = 1 + A * lat;
    int act[AM];
    float4 c[AM];
#pragma unroll
    for (int j = 0; j < AM; ++j) {
      act[j] = root ? rleg[j] : j;
      c[j] = j < n ? cs[base + act[j]] : make_float4(0.0f, 0.0f, __int_as_float(-1), __int_as_float(0));
    }
    const float2 q = nq[lat];
    const int total_v = __float_as_int(q.y);
    float mean_q;
    if (is_root && total_v > 0)
      mean_q = q.x / (float)total_v;
    else
      mean_q = (parent_q + q.x) / (float)(total_v + 1);
    is_root = 0;
    parent_q = mean_q;
    float vu = mm_normalize(mm, mean_q);
    if (vu < 0) vu = 0;
    if (vu > 1) vu = 1;
    float sc[AM];
    float M = -INFINITY;
#pragma unroll
    for (int j = 0; j < AM; ++j) {
      sc[j] = c[j].x + (__float_as_int(c[j].w) ? c[j].y : vu);
      if (j < n) M = fmaxf(M, sc[j]);
    }
    int r = 0;
#pragma unroll
    for (int j = AM - 1; j >= 0; --j)
      if (j < n && sc[j] == M) r = j;
    const float thr = M - 0.000001f;
    unsigned mask = 1u << r;
#pragma unroll
    for (int j = 1; j < AM; ++j)
      if (j < n && j > r && sc[j] >= thr) mask |= 1u << j;
    const int nl = __popc(mask);
    if (CLASSIFY && nl > 1) {
      bool all_leaves = true;
#pragma unroll
      for (int j = 0; j < AM; ++j)
        if (((mask >> j) & 1u) && __float_as_int(c[j].z) >= 0) all_leaves = false;
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = mask;
      Descent d;
      d.len = len + 1;
      d.x = lat;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    int jsel = r;
    if (!CLASSIFY) {
      const uint32_t rr = draw(len);
      int kk = (int)(rr % (uint32_t)nl);
      unsigned m_ = mask;
      for (; kk > 0; --kk) m_ &= m_ - 1;
      jsel = __ffs(m_) - 1;
    }
    int action = act[0], nlat = __float_as_int(c[0].z);
#pragma unroll
    for (int j = 1; j < AM; ++j)
      if (jsel == j) {
        action = act[j];
        nlat = __float_as_int(c[j].z);
      }
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    node = base + action;
    last_action = action;
    if (lane == 0) {
      t.path_act[len] = action;
      t.path[len + 1] = node;
    }
    ++len;
    plat = lat;
    lat = nlat;
  }
  Descent d;
  d.len = len;
  d.x = plat;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

// descend_small for exactly two actions, written for the shortest dependent chain per level. The
// terms phase precomputes each node's walk-independent outcome (dec[latent], a2_decision); where
// it is known the level is a pointer chase — the next node's terms are read while this level's
// mean-q division (needed further down only) completes. Only a node with an unvisited child waits
// for its normalised mean-q. The normaliser's divisor is fixed per walk (mm_normalize's branches
// become one division); same float operations as descend_terms, so the same bits.
__device__ __forceinline__ float mm_norm_fixed(bool scale, float lo, float div, float v) {
  return scale ? (v - lo) / div : v;
}

// OPT (experiments): bit 0 collects the path in lanes (one store at the end instead of two LDS
// stores per level), bit 1 reads the next level's node data before this level's mean-q division.
template <bool CLASSIFY, typename Draw, int OPT = 0>
__device__ inline Descent descend_a2(const TreeView &t, const float2 *nq, const int *dec, const float4 *cs, float4 mm,
                                     int vtp, int players, const int *rleg, int nleg, Draw draw, TieInfo *tie,
                                     WalkState *resume = nullptr, WalkState *at_tie = nullptr,
                                     float2 *chain = nullptr) {
  const int lane = threadIdx.x & 63;
  const float delta = mm.x - mm.y;
  const bool scale = delta > 0;
  const float div = (delta < mm.z) ? mm.z : delta;
  const float lo = mm.y;
  WalkState w0 = resume ? *resume : walk_start(t, vtp);
  int node = w0.node, len = w0.len, last_action = w0.last_action, plat = w0.plat, lat = w0.lat;
  float parent_q = w0.parent_q;
  bool is_root = w0.is_root;
  vtp = w0.vtp;
  if (lane == 0 && !resume) t.path[0] = 0;
  if (CLASSIFY) tie->status = 0;
  const int dmax = t.depth_cap - 1;
  const bool lanes_path = (OPT & 1) && t.depth_cap <= 64;
  const int len0 = len;
  int pnode = 0, pact = 0;
  auto flush = [&]() {
    if (lanes_path) {
      if (lane > len0 && lane <= len) t.path[lane] = pnode;
      if (lane >= len0 && lane < len) t.path_act[lane] = pact;
    }
  };
  int a0 = 0, a1 = 0, n = 2;
  float4 c0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), c1 = c0;
  float2 q = make_float2(0.0f, 0.0f);
  int dl = 2;
  auto fetch = [&](int nd, int lt) {
    const bool root = nd == 0;  // (only the first level of a walk from the root)
    a0 = root ? rleg[0] : 0;
    a1 = root ? rleg[1] : 1;
    n = root ? nleg : 2;
    const int base = 1 + 2 * lt;
    c0 = cs[base + a0];
    c1 = cs[base + (n > 1 ? a1 : a0)];
    q = nq[lt];
    dl = dec[lt];
  };
  if ((OPT & 2) && lat >= 0) fetch(node, lat);
  // OPT & 4: the mean-q chain is evaluated lazily — a level whose outcome is known only records
  // its (total_q, total_v) in chain[]; the divisions run (in level order, the same operations)
  // when a level needs its normalised mean-q or a tie needs parent_q
  const bool lazy = (OPT & 4) && chain != nullptr;
  const bool root0 = is_root;
  int pend = len;
  auto settle = [&](int upto) {
    for (int l = pend; l < upto; ++l) {
      const float2 cq = chain[l];
      const int tv = __float_as_int(cq.y);
      parent_q = (l == len0 && root0 && tv > 0) ? cq.x / (float)tv : (parent_q + cq.x) / (float)(tv + 1);
    }
    pend = upto > pend ? upto : pend;
  };
  while (lat >= 0 && len < dmax) {
    if (!(OPT & 2)) fetch(node, lat);
    const int base = 1 + 2 * lat;
    const int total_v = __float_as_int(q.y);
    const float qx = q.x;
    int jsel = dl;
    bool tie2 = dl == 3;
    float mean_q = 0.0f;
    if (lazy && (dl == 2 || (CLASSIFY && dl == 3))) settle(len);
    const bool rootq = (lazy ? (len == len0 && root0) : is_root) && total_v > 0;
    if ((!(OPT & 2) && !lazy) || dl == 2) mean_q = rootq ? qx / (float)total_v : (parent_q + qx) / (float)(total_v + 1);
    if (dl == 2) {
      float vu = mm_norm_fixed(scale, lo, div, mean_q);
      if (vu < 0) vu = 0;
      if (vu > 1) vu = 1;
      const float s0 = c0.x + (__float_as_int(c0.w) ? c0.y : vu);
      const float s1 = c1.x + (__float_as_int(c1.w) ? c1.y : vu);
      const float M = fmaxf(s0, s1);
      jsel = (s0 == M) ? 0 : 1;
      tie2 = jsel == 0 && s1 >= M - 0.000001f;
    }
    if (CLASSIFY && tie2) {
      if (at_tie) {
        at_tie->node = node; at_tie->lat = lat; at_tie->len = len; at_tie->plat = plat;
        at_tie->last_action = last_action; at_tie->is_root = is_root; at_tie->vtp = vtp; at_tie->parent_q = parent_q;
      }
      flush();
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      const bool all_leaves = __float_as_int(c0.z) < 0 && __float_as_int(c1.z) < 0;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = 3ull;
      Descent d;
      d.len = len + 1;
      d.x = lat;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    if (!CLASSIFY && tie2) jsel = (int)(draw(len) % 2u);
    const int action = jsel ? a1 : a0;
    const int nlat = __float_as_int(jsel ? c1.z : c0.z);
    const int nnode = base + action;
    if (OPT & 2) {
      if (nlat >= 0) fetch(nnode, nlat);
      if (dl != 2) mean_q = rootq ? qx / (float)total_v : (parent_q + qx) / (float)(total_v + 1);
    }
    is_root = false;
    if (!lazy) {
      parent_q = mean_q;
    } else if (dl == 2) {
      parent_q = mean_q;
      pend = len + 1;
    } else if (lane == 0) {
      chain[len] = make_float2(qx, __int_as_float(total_v));
    }
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    node = nnode;
    last_action = action;
    if (lanes_path) {
      pact = lane == len ? action : pact;
      pnode = lane == len + 1 ? node : pnode;
    } else if (lane == 0) {
      t.path_act[len] = action;
      t.path[len + 1] = node;
    }
    ++len;
    plat = lat;
    lat = nlat;
  }
  flush();
  Descent d;
  d.len = len;
  d.x = plat;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

// Depth speculation for a classification walk stopped at a tie between children of which one is
// expanded (status 2, A == 2): lane `pattern` continues the walk from the tie's state taking, at the
// i-th tie on its way, the child that draw parity bit i of `pattern` selects (rr % 2 picks legal
// position 0 or 1); returns that walk's depth (Descent::len), or -1 when it meets more than 6 ties.
// If all 64 patterns give one depth, the root's draw count is known before any of its draw values:
// it is published at once and the path is resolved after the look-back (same walk, same bits).
// Same per-level operations as descend_a2.
// (LZM_RES_SPEC_PATH: *choice gets bit l = the legal position taken at level w.len + l, *ties bit l
// when that level was a tie decided by the pattern, *leaf_tie the offset of a final tie between two
// unexpanded children (its draw picks the leaf; -1: none); *choice = ~0u when the walk is longer than
// 31 levels past w.len. The path of a walk is then its choice bits: the look-back's draw parities
// select the lane whose pattern matches, and the path is a pointer chase without the scores.)
__device__ inline int speculate_depth_a2(const TreeView &t, const float2 *nq, const int *dec, const float4 *cs,
                                         float4 mm, const int *rleg, int nleg, const WalkState &w, int pattern,
                                         uint32_t *choice = nullptr, uint32_t *ties = nullptr, int *leaf_tie = nullptr) {
  uint32_t ch = 0u, tm = 0u;
  if (leaf_tie) *leaf_tie = -1;
  const float delta = mm.x - mm.y;
  const bool scale = delta > 0;
  const float div = (delta < mm.z) ? mm.z : delta;
  const float lo = mm.y;
  int node = w.node, len = w.len, lat = w.lat, used = 0;
  bool is_root = w.is_root;
  float parent_q = w.parent_q;
  const int dmax = t.depth_cap - 1;
  while (lat >= 0 && len < dmax) {
    const bool root = node == 0;
    const int a0 = root ? rleg[0] : 0, a1 = root ? rleg[1] : 1, n = root ? nleg : 2;
    const int base = 1 + 2 * lat;
    const float4 c0 = cs[base + a0];
    const float4 c1 = cs[base + (n > 1 ? a1 : a0)];
    const float2 q = nq[lat];
    const int dl = dec[lat];
    const int total_v = __float_as_int(q.y);
    const float mean_q = (is_root && total_v > 0) ? q.x / (float)total_v : (parent_q + q.x) / (float)(total_v + 1);
    int jsel = dl;
    bool tie2 = dl == 3;
    if (dl == 2) {
      float vu = mm_norm_fixed(scale, lo, div, mean_q);
      if (vu < 0) vu = 0;
      if (vu > 1) vu = 1;
      const float s0 = c0.x + (__float_as_int(c0.w) ? c0.y : vu);
      const float s1 = c1.x + (__float_as_int(c1.w) ? c1.y : vu);
      const float M = fmaxf(s0, s1);
      jsel = (s0 == M) ? 0 : 1;
      tie2 = jsel == 0 && s1 >= M - 0.000001f;
    }
    const int off = len - w.len;
    if (tie2) {
      if (__float_as_int(c0.z) < 0 && __float_as_int(c1.z) < 0) {  // either way a leaf
        if (choice) { *choice = off < 31 ? ch : ~0u; *ties = tm; *leaf_tie = off; }
        return len + 1;
      }
      if (used == 6) return -1;
      jsel = (pattern >> used) & 1;
      ++used;
      if (off < 31) tm |= 1u << off;
    }
    if (off < 31) ch |= (uint32_t)jsel << off;
    is_root = false;
    parent_q = mean_q;
    node = base + (jsel ? a1 : a0);
    lat = __float_as_int(jsel ? c1.z : c0.z);
    ++len;
  }
  if (choice) { *choice = len - w.len <= 31 ? ch : ~0u; *ties = tm; }
  return len;
}

// descend_a2 with the walk state cut to what a decided level needs: the root level runs through
// descend_a2's general body (legal list, root mean-q rule); below it a level whose outcome is
// known (dec 0 / 1) is a pointer chase plus the mean-q division for the next level, and any other
// level (an unvisited child or a tie) hands the walk back to descend_a2 at that level's state
// (same operations either way, so the same bits). vtp flips per level are applied at the end.
template <bool CLASSIFY, typename Draw>
__device__ inline Descent descend_a2f(const TreeView &t, const float2 *nq, const int *dec, const float4 *cs, float4 mm,
                                      int vtp, int players, const int *rleg, int nleg, Draw draw, TieInfo *tie,
                                      WalkState *at_tie = nullptr) {
  const int lane = threadIdx.x & 63;
  // root level: the general body for one level
  WalkState w = walk_start(t, vtp);
  if (w.lat < 0 || t.depth_cap <= 1) return descend_a2<CLASSIFY>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, draw, tie,
                                                                  nullptr, at_tie);
  {
    const int dl = dec[w.lat];
    if (dl >= 2) return descend_a2<CLASSIFY>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, draw, tie, nullptr, at_tie);
    const float2 q = nq[w.lat];
    const int action = rleg[dl];
    const float4 c = cs[1 + 2 * w.lat + action];
    const int tv = __float_as_int(q.y);
    w.parent_q = tv > 0 ? q.x / (float)tv : (0.0f + q.x) / (float)(tv + 1);
    if (lane == 0) {
      t.path[0] = 0;
      t.path_act[0] = action;
      t.path[1] = 1 + 2 * w.lat + action;
    }
    w.node = 1 + 2 * w.lat + action;
    w.last_action = action;
    w.plat = w.lat;
    w.lat = __float_as_int(c.z);
    w.len = 1;
    w.is_root = 0;
  }
  // non-root levels: two children at legal positions 0 / 1
  int lat = w.lat, node = w.node, len = w.len, plat = w.plat, last_action = w.last_action;
  float parent_q = w.parent_q;
  const int dmax = t.depth_cap - 1;
  int dl = 2;
  while (lat >= 0 && len < dmax) {
    dl = dec[lat];
    if (dl >= 2) break;
    const float2 q = nq[lat];
    const float4 c = cs[1 + 2 * lat + dl];
    const int nnode = 1 + 2 * lat + dl;
    if (lane == 0) {
      t.path_act[len] = dl;
      t.path[len + 1] = nnode;
    }
    parent_q = (parent_q + q.x) / (float)(__float_as_int(q.y) + 1);
    last_action = dl;
    node = nnode;
    plat = lat;
    lat = __float_as_int(c.z);
    ++len;
  }
  if (players > 1 && (len & 1)) vtp = (vtp == 1) ? 2 : 1;
  if (lat >= 0 && len < dmax) {
    // an undecided level: continue with the general body from this level's state
    WalkState r;
    r.node = node; r.lat = lat; r.len = len; r.plat = plat; r.last_action = last_action; r.is_root = 0;
    r.vtp = vtp; r.parent_q = parent_q;
    return descend_a2<CLASSIFY>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, draw, tie, &r, at_tie);
  }
  if (CLASSIFY) tie->status = 0;
  Descent d;
  d.len = len;
  d.x = plat;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

// descend_terms by one lane: the reference's sequential tie-list scan (cselect_child,
// cnode.cpp:551-596) over the precomputed terms, no cross-lane operations.
template <bool CLASSIFY, typename Draw>
__device__ inline Descent descend_terms_lane(const TreeView &t, const float2 *nq, const float4 *cs, float4 mm, int vtp,
                                             int players, Draw draw, TieInfo *tie) {
  int node = 0, is_root = 1, len = 0, last_action = -1, plat = -1;
  float parent_q = 0.0f;
  int lat = t.meta[0].latent;
  t.path[0] = 0;
  if (CLASSIFY) tie->status = 0;
  while (lat >= 0 && len < t.depth_cap - 1) {
    const int n = legal_n(t, 0, node);
    const int base = 1 + t.A * lat;
    const float2 q = nq[lat];
    const int total_v = __float_as_int(q.y);
    float mean_q;
    if (is_root && total_v > 0)
      mean_q = q.x / (float)total_v;
    else
      mean_q = (parent_q + q.x) / (float)(total_v + 1);
    is_root = 0;
    parent_q = mean_q;
    float vu = mm_normalize(mm, mean_q);
    if (vu < 0) vu = 0;
    if (vu > 1) vu = 1;
    float max_score = kFloatMin;
    uint64_t mask = 0;
    bool all_leaves = true;
    for (int j = 0; j < n; ++j) {
      const float4 c = cs[base + legal_at(t, 0, node, j)];
      const float score = c.x + (__float_as_int(c.w) ? c.y : vu);
      if (max_score < score) {
        max_score = score;
        mask = 1ull << j;
        all_leaves = __float_as_int(c.z) < 0;
      } else if (score >= max_score - 0.000001f) {
        mask |= 1ull << j;
        all_leaves = all_leaves && __float_as_int(c.z) < 0;
      }
    }
    const int nl = __popcll(mask);
    if (CLASSIFY && nl > 1) {
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      tie->status = all_leaves ? 1 : 2;
      tie->level = len;
      tie->mask = mask;
      Descent d;
      d.len = len + 1;
      d.x = lat;
      d.action = -1;
      d.vtp = vtp;
      d.leaf = -1;
      return d;
    }
    const uint32_t rr = CLASSIFY ? 0u : draw(len);
    int kk = (int)(rr % (uint32_t)nl);
    uint64_t mm_ = mask;
    for (; kk > 0; --kk) mm_ &= mm_ - 1;
    const int jsel = __ffsll((long long)mm_) - 1;
    const int action = legal_at(t, 0, node, jsel);
    if (players > 1) vtp = (vtp == 1) ? 2 : 1;
    node = base + action;
    last_action = action;
    t.path_act[len] = action;
    t.path[len + 1] = node;
    ++len;
    plat = lat;
    lat = __float_as_int(cs[node].z);
  }
  Descent d;
  d.len = len;
  d.x = plat;
  d.action = last_action;
  d.vtp = vtp;
  d.leaf = node;
  return d;
}

// NR rows of a 128 x 128 layer (inputs x + r * 128): each weight read once for all rows.
#ifndef LZM_RES_STAGE_WD1
#define LZM_RES_STAGE_WD1 1
#endif
struct NoSide {
  __device__ __forceinline__ void operator()(int) const {}
};
// side(j) runs at the top of slot j: a weight prefetch spread over the layer, one or two buffer
// loads per slot, instead of a burst that stalls the wave at issue (the texture path takes a
// 1 KiB wave-load per 16 cycles and four waves share it)
template <int NR, typename WF, typename SF = NoSide>
__device__ __forceinline__ void dense128n(const float *x, WF w, float *z, SF side = SF()) {
#if LZM_RES_D4
  const int e = threadIdx.x & 7;
  float4 xv[NR][4];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[r][j] = reinterpret_cast<const float4 *>(x + r * kRRow)[4 * e + (e >> 2) + j];
  float a[NR][4][4];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) a[r][c][0] = a[r][c][1] = a[r][c][2] = a[r][c][3] = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      side(4 * j + c);
      const float4 q = w(4 * j + c);
#pragma unroll
      for (int r = 0; r < NR; ++r) fma4(xv[r][j], q, a[r][c]);
    }
#pragma unroll
  for (int r = 0; r < NR; ++r)
    z[r] = reduce_d4((a[r][0][0] + a[r][0][1]) + (a[r][0][2] + a[r][0][3]),
                     (a[r][1][0] + a[r][1][1]) + (a[r][1][2] + a[r][1][3]),
                     (a[r][2][0] + a[r][2][1]) + (a[r][2][2] + a[r][2][3]),
                     (a[r][3][0] + a[r][3][1]) + (a[r][3][2] + a[r][3][3]));
#else
  const int p = threadIdx.x & 1;
  float a[NR][4];
#pragma unroll
  for (int r = 0; r < NR; ++r) a[r][0] = a[r][1] = a[r][2] = a[r][3] = 0.0f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    side(j);
    const float4 q = w(j);
#pragma unroll
    for (int r = 0; r < NR; ++r) fma4(reinterpret_cast<const float4 *>(x + r * kRRow)[kRHalf4 * p + j], q, a[r]);
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const float h = (a[r][0] + a[r][1]) + (a[r][2] + a[r][3]);
    z[r] = h + dpp_f<0xB1>(h);
  }
#endif
}

// NH supports decoded together (z[h] = this lane's logits of support h, see support_logits):
// the reductions of support_decode sharing its two barriers. red: 12 * NH floats of LDS.
template <int NH>
__device__ __forceinline__ void support_decode_n(const float (*z)[3], float *red, float *out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool ok2 = tid < 2 * kRTail && !(tid & 1);
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    float m = fmaxf(z[h][0], z[h][1]);
    if (ok2) m = fmaxf(m, z[h][2]);
    m = wave_max_dpp(m);
    if (lane == 0) red[4 * h + wid] = m;
  }
  __syncthreads();
  const float half = (float)((kRV - 1) / 2);
  const float j0 = (float)tid - half, j1 = (float)(kRT + tid) - half, j2 = (float)(2 * kRT + (tid >> 1)) - half;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const float M = fmaxf(fmaxf(red[4 * h], red[4 * h + 1]), fmaxf(red[4 * h + 2], red[4 * h + 3]));
    const float e0 = expf(z[h][0] - M), e1 = expf(z[h][1] - M), e2 = ok2 ? expf(z[h][2] - M) : 0.0f;
    float se = (e0 + e1) + e2, sj = (e0 * j0 + e1 * j1) + e2 * j2;
    se = wave_sum(se);
    sj = wave_sum(sj);
    if (lane == 0) {
      red[4 * NH + 8 * h + wid] = se;
      red[4 * NH + 8 * h + 4 + wid] = sj;
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const float *q = red + 4 * NH + 8 * h;
    out[h] = h_inverse(((q[4] + q[5]) + (q[6] + q[7])) / ((q[0] + q[1]) + (q[2] + q[3])));
  }
}

// A parity-mode tie among unexpanded children resolved with its draw rr: the chosen child ends
// the path (cselect_child's list[rand() % len], cnode.cpp:592); one thread.
__device__ inline void resolve_tie(const TreeView &t, int A, int lvl, unsigned long long m, uint32_t rr, int *act) {
  int kk = (int)(rr % (uint32_t)__popcll(m));
  for (; kk > 0; --kk) m &= m - 1;
  const int jsel = __ffsll((long long)m) - 1;
  const int parent = t.path[lvl];
  const int action = legal_at(t, 0, parent, jsel);
  t.path_act[lvl] = action;
  t.path[lvl + 1] = 1 + A * t.meta[parent].latent + action;
  *act = action;
}

// Sum of the draw counts published by workgroups < g for simulation k, by the whole workgroup: one
// flag per thread (every poll in flight at once, not one round per 64 predecessors), reduced
// through LDS (part: kRWaves ints). Bounded spin; ends with a barrier.
__device__ inline int lookback_sum(const SearchArgs &p, int k, int g, int G, unsigned long long epoch, int *part) {
  const int lane = threadIdx.x & 63;
  int sum = 0;
  for (int q = threadIdx.x; q < g; q += kRT) {
    unsigned long long v;
    long long spins = 0;
    while (true) {
      v = __hip_atomic_load(&p.flags[(size_t)k * G + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((v >> 32) == epoch) break;
      if (++spins > (1ll << 22)) {
        atomicAdd(p.diag, 1);
        v = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    sum += (int)(v & 0xffffffffu);
  }
  sum = xor_sum(sum);
  if (lane == 0) part[threadIdx.x >> 6] = sum;
  __syncthreads();
  return (part[0] + part[1]) + (part[2] + part[3]);
}

// lookback_sum by one wave, for G <= 256 workgroups: lane l polls roots l, l + 64, ... (all
// loads in flight at once), the sum by DPP (exact: float sums of integers < 2^24), no LDS and no
// barrier. Returns the sum in every lane of the calling wave. Every wave of the late draw calls it on
// its own, so a spin timeout is counted in p.diag once per wave that met it, and two waves may then
// disagree on the base; any count invalidates the whole search (lzm_check_errors raises at the result
// getters, the collector and bench.py), so such a search is never used.
__device__ inline int lookback_sum_w0(const SearchArgs &p, int k, int g, int G, unsigned long long epoch) {
  const int lane = threadIdx.x & 63;
  const unsigned long long ok = epoch << 32;  // a published flag of depth 0
  unsigned long long v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = lane + 64 * j;
    v[j] = q < g ? __hip_atomic_load(&p.flags[(size_t)k * G + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ok;
  }
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = lane + 64 * j;
    long long spins = 0;
    while ((v[j] >> 32) != epoch) {
      if (++spins > (1ll << 22)) {
        atomicAdd(p.diag, 1);
        v[j] = ok;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v[j] = __hip_atomic_load(&p.flags[(size_t)k * G + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    sum += (float)(int)(v[j] & 0xffffffffu);
  }
  return (int)wave_sum(sum);
}

// NR = 2 (parity mode): the network carries a second, speculative row for two-way leaf ties.
// SMODE: the selection mode at compile time (-1: n.select_mode at run time, experiments); RNG:
// 0 glibc, 1 Philox, -1 p.fast at run time; STAMPS: phase stamps compiled in (LZM_PHASE_TIMING).
// Production launches fix all three, so the unused paths cost neither code nor registers.
// The kernel's dynamic LDS plan (float offsets from the dynamic base): the two LDS weight layers
// first (their slot addresses become instruction immediates), then the tree slice, the selection
// tables and the optional pUCT visit table. cap / lut_n / depth_cap: the handle's capacities;
// S: simulations the selection tables hold. (A compile-time plan for the production handle, which
// frees ~45 scalar registers of offsets, measured even: the scalar spills are not on the path.)
// static LDS of the kernel: activations (two rows), biases, scalars (below 2 KiB)
constexpr int kResStaticBytes = (kRRow + 4 * kRRow + 2 * (4 * kRRow + kRF + 2 * kRF + kRMaxA) + kResBiasFloats) * 4 + 2048;
constexpr int kResMaxBytes = 160 * 1024 - kResStaticBytes;
__host__ __device__ constexpr int res_round4(int x) { return (x + 3) & ~3; }
__host__ __device__ constexpr ResPlan res_plan(int cap, int lut_n, int depth_cap, int S, int A) {
  ResPlan q{};
  int o = 0;
  q.wd1 = o; o += kRSlotsD * kRT * 4;
  q.wd2 = o; o += kRSlotsD * kRT * 4;
  q.stat = o; o += cap * 4;
  q.meta = o; o += cap * 4;
  q.lut = o; o += res_round4(2 * lut_n);
  q.legal = o; o += res_round4(A + 1);
  q.val = o; o += res_round4(cap);
  q.path = o; o += res_round4(depth_cap);
  q.pact = o; o += res_round4(depth_cap);
  q.act = o; o += A * kRHid;
  q.l2n = o; o += res_round4(S + 2);
  q.nq = o; o += res_round4(2 * (S + 2));
  q.cs = o; o += 4 * cap;
  q.dec = o; o += res_round4(S + 2);
  q.misc = o; o += res_round4(S + 32);
  const int tri = res_round4(lut_n * (lut_n + 1) / 2);
  q.pbt = o;
  q.pbt_rows = ((o + tri) * 4 <= kResMaxBytes && tri <= 8192) ? lut_n : 0;
  if (q.pbt_rows) o += tri;
  q.floats = o;
  return q;
}

template <int NR, int SMODE, int RNG, bool STAMPS>
__global__ __launch_bounds__(kRT) __attribute__((amdgpu_waves_per_eu(1, 1))) void search_res_kernel(SearchArgs p, ResNet n) {
  if (!STAMPS) p.phase = nullptr;
  if (RNG >= 0) p.fast = RNG;
  const ResPlan L = n.plan;
  if (SMODE >= 0) n.select_mode = SMODE;
  if (SMODE == 4 && RNG == 0 && !STAMPS) n.spec_depth = 1;  // production parity kernel
  extern __shared__ float4 smem4[];
  float *smem = reinterpret_cast<float *>(smem4);
  const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x, lane = tid & 63, wid = tid >> 6;
  const int B = p.B, A = p.A;
  const int i = g;  // one root per workgroup
  unsigned long long stamp_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;
  unsigned long long isub_ = stamp_;  // init sub-stamps (diagnostics)
#define LZM_ISTAMP(n)                                                      \
  do {                                                                     \
    if (p.phase && tid == 0) {                                             \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();       \
      s_phase[n] += (now_ - isub_) * (unsigned long long)p.S;              \
      isub_ = now_;                                                        \
    }                                                                      \
  } while (0)

  __shared__ uint32_t s_z0[31];
  __shared__ int s_players, s_epoch, s_x, s_act, s_status, s_tlevel, s_vtp;
  __shared__ int s_len[1], s_part[kRWaves], s_nlat;
  __shared__ unsigned long long s_tmask;
  __shared__ WalkState s_walk;
  __shared__ float4 s_mm;
  __shared__ float s_red[12 * 2 * NR];
  __shared__ uint32_t s_dwin[64];  // LZM_RES_DWIN2: draw sums at stream positions s_dlo + 0..63
  __shared__ int s_dlo, s_base_prev;
  if (tid == 0) { s_dlo = -1000000; s_base_prev = 0; }
  __shared__ uint64_t s_exptab[32];  // glibc_expf's table: expand reads it from LDS (no vmcnt wait
                                     // on the weight prefetch in flight)
  if (threadIdx.x < 32) s_exptab[threadIdx.x] = kExp2fTab[threadIdx.x];
  __shared__ unsigned long long s_phase[64];
  if (p.phase && tid < 64) s_phase[tid] = 0ull;
  unsigned long long s_wait = 0ull;  // (thread 0) look-back wait cycles, diagnostics

  // ---- tree slice into LDS (node records, value cache, pUCT tables, legal list, path)
  TreeView t;
  t.A = A; t.cap = p.cap; t.lut_n = p.lut_n; t.depth_cap = p.depth_cap; t.B = 1;
  t.path = reinterpret_cast<int32_t *>(smem + L.path);
  t.path_act = reinterpret_cast<int32_t *>(smem + L.pact);
  t.pathlen = s_len;
  {
    NodeStat *ls = reinterpret_cast<NodeStat *>(smem + L.stat);
    NodeMeta *lm = reinterpret_cast<NodeMeta *>(smem + L.meta);
    float2 *llut = reinterpret_cast<float2 *>(smem + L.lut);
    int32_t *llegal = reinterpret_cast<int32_t *>(smem + L.legal);
    float *lval = smem + L.val;
    for (int e = tid; e < p.cap; e += kRT) {
      const NodeStat s = p.stat[(size_t)e * B + i];
      ls[e] = s;
      lm[e] = p.meta[(size_t)e * B + i];
      lval[e] = node_value(s);
    }
    for (int e = tid; e < p.lut_n; e += kRT) llut[e] = p.lut[e];
    float *lpbt = smem + L.pbt;
    build_pbt(p.lut, p.pbt_rows, lpbt, tid, kRT);
    for (int e = tid; e < A; e += kRT) llegal[e] = p.legal[(size_t)i * A + e];
    if (tid == 0) llegal[A] = p.nlegal[i];
    t.stat = ls; t.meta = lm; t.lut = llut; t.legal = llegal; t.nlegal = llegal + A; t.val = lval;
    t.pbt = p.pbt_rows ? lpbt : nullptr;
  }
  LZM_ISTAMP(24);
  // latent -> node map of the expanded nodes (children of latent L sit at 1 + A L)
  int *L2N = reinterpret_cast<int *>(smem + L.l2n);
  float2 *NQ = reinterpret_cast<float2 *>(smem + L.nq);
  int *DEC = reinterpret_cast<int *>(smem + L.dec);
  float4 *CS = reinterpret_cast<float4 *>(smem + L.cs);
  // A search starts from prepared roots: only the root is expanded, with latent 0 (cnode.cpp:
  // 301-358); simulation k gives its leaf latent k + 1. (Nodes past the root's children may hold a
  // previous search's records: never scan them.)
  for (int e = tid; e < p.S + 2; e += kRT) L2N[e] = e == 0 ? 0 : -1;
  if (tid == 0) s_nlat = 1;
  if (tid == 0) {
    s_mm = p.mm_fresh ? make_float4(kFloatMin, kFloatMax, p.mm_delta, 0.0f) : p.minmax[i];
    s_vtp = p.vtp_in[i];
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wid == 0) {
    // players: 2 unless every root's to_play is -1 (max over the batch), by wave 0 with all its
    // loads in flight (a serial loop over B was ~30 K cycles of the launch)
    int m = INT_MIN;
    for (int q = lane; q < B; q += 64) m = max(m, p.vtp_in[q]);
    m = xor_max(m);
    if (lane == 0) s_players = (m == -1) ? 1 : 2;
  }
  uint32_t *s_seeds = reinterpret_cast<uint32_t *>(smem + L.misc);
  uint32_t *s_pow = s_seeds + p.S;
  if (p.step_count) {
    const long long c = *p.step_count;  // (read before the last workgroup's increment below)
    for (int e = tid; e < p.S; e += kRT) s_seeds[e] = (uint32_t)((p.step_base + c * (long long)p.S + e) % 1000000ll);
  } else {
    for (int e = tid; e < p.S; e += kRT) s_seeds[e] = p.seeds[e];
  }
  if (!p.fast)
    for (int e = tid; e < 31; e += kRT) s_pow[e] = p.pow16807[e];

  LZM_ISTAMP(25);
  // ---- network residency: LDS layers, action rows, register layers and biases
  // activations and biases at static LDS addresses: lane-dependent addresses then share a few base
  // registers and fold the arrays' offsets into the instructions' immediates
  // T1 / NL hold two rows even at NR = 1: the two candidates of a leaf tie run the dynamics
  // layers side by side while the draw offset is still unknown (see the simulation loop)
  __shared__ float4 s_acts[(kRRow + 4 * kRRow + NR * (4 * kRRow + kRF + 2 * kRF + kRMaxA)) / 4];
  __shared__ float4 s_bias[kResBiasFloats / 4];
  float *X0 = reinterpret_cast<float *>(s_acts), *T1 = X0 + kRRow, *NL = T1 + 2 * kRRow, *T2 = NL + 2 * kRRow,
        *T3 = T2 + NR * kRRow, *U2 = T3 + NR * kRRow, *U3 = U2 + NR * kRRow, *RHo = U3 + NR * kRRow,
        *HV = RHo + NR * kRF, *LG = HV + NR * 2 * kRF;
  float *ACT = smem + L.act;
  const float4 *WD1 = reinterpret_cast<const float4 *>(smem + L.wd1);
  const float4 *WD2 = reinterpret_cast<const float4 *>(smem + L.wd2);
  {
    // the two LDS layers, each thread's 16 + 16 slots loaded before any is stored (one round trip
    // per block instead of one per slot: the registers are free before the weights arrive)
    float4 st[kRSlotsD];
    res_fetch<kRSlotsD>(res_blk4(n, kRbD + 1), st);
#pragma unroll
    for (int j = 0; j < kRSlotsD; ++j) reinterpret_cast<float4 *>(smem + L.wd1)[j * kRT + tid] = st[j];
    res_fetch<kRSlotsD>(res_blk4(n, kRbD + 2), st);
#pragma unroll
    for (int j = 0; j < kRSlotsD; ++j) reinterpret_cast<float4 *>(smem + L.wd2)[j * kRT + tid] = st[j];
  }
  for (int e = tid; e < A * kRHid; e += kRT) ACT[e] = res_blk(n, kRbAct, A)[e];
  LZM_ISTAMP(26);
  float4 wD3[kRSlotsD], wD4[kRSlotsD], wRS[kRSlotsS], wRH[kRSlotsRH], wVPH[kRSlotsVPH], wPO[1];
  res_fetch<kRSlotsD>(res_blk4(n, kRbD + 3), wD3);
  res_fetch<kRSlotsD>(res_blk4(n, kRbD + 4), wD4);
  res_fetch<kRSlotsS>(res_blk4(n, kRbRS), wRS);
  res_fetch<kRSlotsRH>(res_blk4(n, kRbRH), wRH);
  res_fetch<kRSlotsVPH>(res_blk4(n, kRbVPH), wVPH);
  res_fetch<kRSlotsPO>(res_blk4(n, kRbPO), wPO);
  const int cD = d_col(), pD = tid & 1, cRH = tid >> 3, pRH = tid & 7, cVP = tid >> 2, pVP = tid & 3, cPO = tid >> 3;
  LZM_ISTAMP(27);
  // biases live in LDS (registers are the scarce resource): the bias blocks are contiguous
  float *BB = reinterpret_cast<float *>(s_bias);
  {
    constexpr int kNB = (kResBiasFloats + kRT - 1) / kRT;
    float bv[kNB];
    const float *bsrc = res_blk(n, kRbBD, A);
#pragma unroll
    for (int j = 0; j < kNB; ++j) bv[j] = j * kRT + tid < kResBiasFloats ? bsrc[j * kRT + tid] : 0.0f;
#pragma unroll
    for (int j = 0; j < kNB; ++j)
      if (j * kRT + tid < kResBiasFloats) BB[j * kRT + tid] = bv[j];
  }
  const float *BD = BB, *BRH = BD + 6 * kRHid, *BVP = BRH + kRF, *BRS = BVP + 2 * kRF,
              *BVS = BRS + ((kRV + 3) & ~3), *BPO = BVS + ((kRV + 3) & ~3);
  // the streamed buffer: fc_dynamics[0] for the first simulation
  float4 P[kRSlotsS];
  res_fetch<kRSlotsD>(res_blk4(n, kRbD), P);
#pragma unroll
  for (int j = kRSlotsD; j < kRSlotsS; ++j) P[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;
  // the root's legal actions in registers (descend_small)
  int rleg[2];
  const int nleg = t.nlegal[0];
#pragma unroll
  for (int j = 0; j < 2; ++j) rleg[j] = j < A ? t.legal[j] : 0;
  LZM_ISTAMP(28);
  LZM_STAMP(10);

  for (int k = 0; k < p.S; ++k) {
    const uint32_t seed = s_seeds[k];
    if (!LZM_RES_SEEDW1 && !p.fast) seed_state_parallel(seed, s_pow, s_z0);
    // ---- selection, part 1: every expanded node's walk-independent pUCT terms (all threads)
    // 0: descend_wave; 1: terms + wave walk; 2: terms + lane walk; 3: descend_slice; 4 (default):
    // terms + descend_small when A <= 2, else as 1
    const int smode = (n.select_mode == 4 && A != 2) ? 1 : n.select_mode;
    if (smode == 1 || smode == 2 || smode == 4) {
      __syncthreads();  // the previous simulation's backup (wave 0) and children (wave 1) are complete
      if (smode == 4)
        precompute_terms_a2(t, s_nlat + k, L2N, NQ, CS, s_mm, players, p.disc, DEC, rleg, nleg);
      else
        precompute_terms(t, s_nlat + k, L2N, NQ, CS, s_mm, players, p.disc, smode == 4 ? DEC : nullptr);
      __syncthreads();
    }
    LZM_STAMP(12);
    if (wid != 0 && k > 0) res_fetch<kRSlotsD>(res_blk4(n, kRbD), P);  // (see the expand)
    if (LZM_RES_SEEDW1 && !p.fast && wid == 1) {  // (the post-walk barrier orders s_z0 for its readers)
      const uint32_t sd = seed == 0 ? 1u : seed;
      if (sd < 0x7fffffffu) {
        if (lane < 31) {
          unsigned long long x = (unsigned long long)sd * s_pow[lane];
          unsigned long long r = (x & 0x7fffffffull) + (x >> 31);
          r = (r & 0x7fffffffull) + (r >> 31);
          if (r >= 0x7fffffffull) r -= 0x7fffffffull;
          s_z0[lane] = (uint32_t)r;
        }
      } else if (lane == 0) {
        glibc_seed_state(seed, s_z0);
      }
    }
    if (LZM_RES_DWIN2 && RNG != 1 && wid == 1) s_dwin[lane] = 0u;  // (the status-2 window's adds follow a barrier)
    // ---- selection, part 2: the walk (wave 0, one lane per child)
    if (wid == 0) {
      const float4 mm = s_mm;
      if (p.fast) {
        auto draw = [seed, i](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)i, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        Descent d;
        if (smode == 4) {
          d = descend_a2f<false>(t, NQ, DEC, CS, mm, s_vtp, players, rleg, nleg, draw, nullptr);
        } else if (smode == 1) {
          d = descend_terms<false>(t, NQ, CS, mm, s_vtp, players, draw, nullptr);
        } else if (smode == 0) {
          d = descend_wave<false, false>(t, 0, 0, 1, mm, players, s_vtp, p.disc, draw, nullptr);
        } else if (lane == 0) {
          d = smode == 2 ? descend_terms_lane<false>(t, NQ, CS, mm, s_vtp, players, draw, nullptr)
                         : descend_slice<false, false>(t, 0, 0, 1, mm, players, s_vtp, p.disc, draw, nullptr);
        }
        if (lane == 0) { s_len[0] = d.len; s_x = d.x; s_act = d.action; s_status = 0; }
      } else {
        TieInfo ti;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        Descent d;
        if (smode == 4) {
          WalkState ws;
          d = descend_a2f<true>(t, NQ, DEC, CS, mm, s_vtp, players, rleg, nleg, nodraw, &ti, &ws);
          LZM_STAMP(13);
          if (lane == 0 && ti.status == 2) s_walk = ws;
        } else if (smode == 1) {
          WalkState ws;
          d = descend_terms<true>(t, NQ, CS, mm, s_vtp, players, nodraw, &ti, nullptr, &ws);
          if (lane == 0 && ti.status == 2) s_walk = ws;
        } else if (smode == 0) {
          d = descend_wave<false, true>(t, 0, 0, 1, mm, players, s_vtp, p.disc, nodraw, &ti);
        } else if (lane == 0) {
          d = smode == 2 ? descend_terms_lane<true>(t, NQ, CS, mm, s_vtp, players, nodraw, &ti)
                         : descend_slice<false, true>(t, 0, 0, 1, mm, players, s_vtp, p.disc, nodraw, &ti);
        }
        if (lane == 0) {
          s_len[0] = d.len; s_x = d.x; s_act = d.action;
          s_status = ti.status; s_tlevel = ti.level; s_tmask = ti.mask;
          // publish this root's draw count at once (its depth is known unless status 2)
          if (ti.status != 2)
            __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#if LZM_RES_EGATHER
      // gather the leaf's parent latent now, by the walking wave, when the walk's x is final (every
      // status but 2): the walk's barrier then also orders the gather (one barrier fewer)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // lane 0's s_status / s_x to the wave
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int stw = __builtin_amdgcn_readfirstlane(s_status);
      const int x0 = __builtin_amdgcn_readfirstlane(s_x);
      if (stw != 2 && lane < kRHid / 4)
        reinterpret_cast<float4 *>(X0)[lane + (lane >= kRHid / 8)] =
            reinterpret_cast<const float4 *>(p.pool + ((size_t)max(x0, 0) * B + i) * kRHid)[lane];
#endif
    }
    __syncthreads();
    LZM_STAMP(0);
    const int status = s_status;
    if (__builtin_expect(status == 2 && (smode == 1 || smode == 4), 0)) {
      // the depth depends on a draw: look back now, then resume the walk at the tie with the draws
      // (exact semantics; the draws of the forced levels above the tie are never read). First
      // (A == 2), when every draw outcome gives the same depth (speculate_depth_a2), publish it at
      // once so that the roots after this one need not wait for this root's look-back (st = 3).
      int st = 2, d0 = -1;
      uint32_t sp_choice = ~0u, sp_ties = 0u;
      int sp_leaf = -1;
      unsigned long long sub_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;
      if (smode == 4 && n.spec_depth && wid == 0) {
        const int de = LZM_RES_SPEC_PATH
                           ? speculate_depth_a2(t, NQ, DEC, CS, s_mm, rleg, nleg, s_walk, lane, &sp_choice, &sp_ties, &sp_leaf)
                           : speculate_depth_a2(t, NQ, DEC, CS, s_mm, rleg, nleg, s_walk, lane);
        d0 = __builtin_amdgcn_readfirstlane(de);
        if (d0 >= 0 && __ballot(de != d0) == 0ull) {
          st = 3;
          if (lane == 0)
            __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)d0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      LZM_SUBSTAMP(20);
      // LZM_RES_DWIN2: wave 0 alone waits for the look-back while wave 1 fills the draw window
      const bool win2 = LZM_RES_DWIN2 && RNG != 1 && smode == 4 && G <= kRT;
      int base = 0;
      if (win2) {
        if (wid == 0) {
          base = lookback_sum_w0(p, k, g, G, epoch);
        } else {
          const int lo = max(s_base_prev - kDwinBack, 0);
          dwin_add_part(p.coef, p.coef_positions, s_z0, lo, s_dwin, wid - 1);
          if (tid == 64) s_dlo = lo;
        }
        __syncthreads();
      } else {
        base = lookback_sum(p, k, g, G, epoch, s_part);
      }
      LZM_SUBSTAMP(21);
      if (wid == 0) {
        if (lane == 0) atomicAdd(p.diag + (st == 2 ? 1 : 2), 1);
        WalkState ws = s_walk;
        // the levels whose draws the resumed walk can read: below the speculated depth (st 3)
        const int hi = st == 3 ? d0 : t.depth_cap;
        bool need = true;
        uint32_t wv = 0u;
        if (win2) {
          bool miss;
          wv = window_draw(p.coef_positions, base, ws.len, hi, s_dwin, s_dlo, &miss);
          need = __ballot(miss) != 0ull;
          if (lane == 0) s_base_prev = base;
          if (p.phase && lane == 0 && need) s_phase[41] += 1;  // window misses (diagnostics)
        }
        if (need) {  // (lane_draws' rows)
          const int q = base + ws.len + lane;
          wv = 0u;
          if (ws.len + lane < hi && q < p.coef_positions) {
            const uint32_t *c = p.coef + (size_t)q * 31;
#pragma unroll
            for (int j = 0; j < 31; ++j) wv += c[j] * s_z0[j];
            wv >>= 1;
          }
        }
        const LaneDraws draw{p.coef, s_z0, p.diag, p.coef_positions, base, ws.len, wv};
        Descent d;
        // LZM_RES_SPEC_PATH: the lane whose pattern agrees with the draws' parities at its tie levels
        // (lane l holds the draw of level ws.len + l); that lane's choice bits are the path
        int m = -1;
        uint32_t pch = 0u;
        if (LZM_RES_SPEC_PATH && st == 3 && smode == 4) {
          const unsigned long long par = __ballot((wv & 1u) != 0u);
          const bool ok = sp_choice != ~0u && ((sp_choice ^ (uint32_t)par) & sp_ties) == 0u;
          const unsigned long long okm = __ballot(ok);
          if (okm) {
            m = __ffsll((long long)okm) - 1;
            pch = (uint32_t)__builtin_amdgcn_readlane((int)sp_choice, m);
            const int lt = __builtin_amdgcn_readlane(sp_leaf, m);
            if (lt >= 0) pch = (pch & ~(1u << lt)) | ((uint32_t)(par >> lt) & 1u) << lt;
          }
        }
        if (m >= 0) {
          int node = ws.node, lat = ws.lat, len = ws.len, plat = ws.plat, last_action = ws.last_action;
          const int dmax = t.depth_cap - 1;
          while (lat >= 0 && len < dmax) {
            const bool root = node == 0;
            const int j = (int)((pch >> (len - ws.len)) & 1u);
            const int action = j ? (root ? rleg[1] : 1) : (root ? rleg[0] : 0);
            const int nnode = 1 + 2 * lat + action;
            const int nlat = __float_as_int(CS[nnode].z);
            if (lane == 0) {
              t.path_act[len] = action;
              t.path[len + 1] = nnode;
            }
            ++len;
            plat = lat;
            lat = nlat;
            node = nnode;
            last_action = action;
          }
          d.len = len;
          d.x = plat;
          d.action = last_action;
          d.vtp = 0;
          d.leaf = node;
        } else if (smode == 4)
          d = descend_a2<false>(t, NQ, DEC, CS, s_mm, s_vtp, players, rleg, nleg, draw, nullptr, &ws);
        else
          d = descend_terms<false>(t, NQ, CS, s_mm, s_vtp, players, draw, nullptr, &ws);
        if (lane == 0) {
          if (st == 3 && d.len != d0) {
            // cannot happen (the speculation walked every draw outcome); counted as an integrity error
            atomicAdd(p.diag, 1);
            atomicAdd(p.diag + 3, 1);
          }
          s_len[0] = d.len; s_x = d.x; s_act = d.action;
          if (st == 2)
            __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (LZM_RES_EGATHER) {  // X0 by this wave (the barrier below orders it)
          const int x0 = __builtin_amdgcn_readfirstlane(d.x);
          if (lane < kRHid / 4)
            reinterpret_cast<float4 *>(X0)[lane + (lane >= kRHid / 8)] =
                reinterpret_cast<const float4 *>(p.pool + ((size_t)max(x0, 0) * B + i) * kRHid)[lane];
        }
      }
      LZM_SUBSTAMP(22);
      __syncthreads();
      LZM_SUBSTAMP(23);
    } else if (status == 2) {
      // the depth depends on a draw: look back now, then walk with the draws (exact semantics)
      const int base = lookback_sum(p, k, g, G, epoch, s_part);
      if (tid == 0) {
        {
          atomicAdd(p.diag + 1, 1);
          const uint32_t *coef = p.coef;
          const int npos = p.coef_positions;
          int32_t *diag = p.diag;
          auto draw = [coef, npos, diag, base](int level) -> uint32_t {
            return glibc_draw(coef, npos, s_z0, base + level, diag);
          };
          Descent d = descend_slice<false, false>(t, 0, 0, 1, s_mm, players, s_vtp, p.disc, draw, nullptr);
          s_len[0] = d.len; s_x = d.x; s_act = d.action;  // (s_status stays: other waves may still read it)
          __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
    }
    LZM_STAMP(1);
    // ---- gather the leaf's parent latent: X0 = pool[x][i] (LZM_RES_EGATHER: already done by the
    // walking wave)
    const bool gathered = LZM_RES_EGATHER && (status != 2 || smode == 1 || smode == 4);
    if (!gathered) {
      if (tid < kRHid / 4)
        reinterpret_cast<float4 *>(X0)[tid + (tid >= kRHid / 8)] =
            reinterpret_cast<const float4 *>(p.pool + ((size_t)max(s_x, 0) * B + i) * kRHid)[tid];
      __syncthreads();
    }
    LZM_STAMP(2);
    unsigned long long sub_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;
    // ---- fc_dynamics[0], latent rows (streamed weights in P): shared by the speculative rows
    const float z0 = dense128(X0, [&](int j) { return P[j]; });
#if LZM_RES_STAGE_WD1
    // the stream buffer is free until the next pair's prefetch: stage fc_dynamics[1]'s LDS slots in
    // it now, so the layer below reads registers (its LDS reads in flight during the action rows)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kRSlotsD; ++j) P[j] = WD1[j * kRT + tid];
#endif
    LZM_SUBSTAMP(16);
    // Rows: row r carries the network for action act_r. A tie between exactly two unexpanded
    // children (status 1) is evaluated speculatively for both (NR = 2) and resolved after the
    // network, when the predecessors' draw counts have long been published; other ties wait here.
    // NR = 1, late draw: a two-way leaf tie runs the two dynamics layers for both candidates (two
    // rows, shared weight reads) and only then waits for the look-back, which by then has mostly
    // been published; the draw picks the next-latent row the rest of the network reads.
    bool spec = false, late = false;
    int act_r[2];
    if (status == 1) {
      const unsigned long long m = s_tmask;
      const int parent = t.path[s_tlevel];
      if (__popcll(m) == 2 && (NR == 2 || n.late_draw)) {
        spec = NR == 2;
        late = NR == 1;
        act_r[0] = legal_at(t, 0, parent, __ffsll((long long)m) - 1);
        act_r[1] = legal_at(t, 0, parent, __ffsll((long long)(m & (m - 1))) - 1);
      } else {
        const int base = lookback_sum(p, k, g, G, epoch, s_part);
        if (tid == 0) resolve_tie(t, A, s_tlevel, m, glibc_draw(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.diag), &s_act);
        __syncthreads();
      }
    }
    if (!spec && !late) act_r[0] = act_r[1] = s_act;
    LZM_SUBSTAMP(17);
    __builtin_amdgcn_sched_barrier(0);
    // + the action's one-hot row, bias, ReLU (muzero_model_mlp.py:188-190)
    if (pD == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
        if (r < NR || late) T1[r * kRRow + rpad(cD)] = fmaxf((z0 + ACT[act_r[r] * kRHid + cD]) + BD[cD], 0.0f);
    }
    __syncthreads();
    LZM_SUBSTAMP(18);
    // ---- fc_dynamics[1] (LDS weights) + latent residual -> next latent
    if (NR == 1 && late) {
      float z[2];
#if LZM_RES_STAGE_WD1
      dense128n<2>(T1, [&](int j) { return P[j]; }, z);
#else
      dense128n<2>(T1, [&](int j) { return WD1[j * kRT + tid]; }, z);
#endif
      LZM_SUBSTAMP(32);
      if (pD == 0) {
#pragma unroll
        for (int r = 0; r < 2; ++r) NL[r * kRRow + rpad(cD)] = fmaxf(z[r] + BD[kRHid + cD], 0.0f) + X0[rpad(cD)];
      }
    } else {
      float z[NR];
#if LZM_RES_STAGE_WD1
      dense128n<NR>(T1, [&](int j) { return P[j]; }, z);
#else
      dense128n<NR>(T1, [&](int j) { return WD1[j * kRT + tid]; }, z);
#endif
      if (pD == 0) {
#pragma unroll
        for (int r = 0; r < NR; ++r) NL[r * kRRow + rpad(cD)] = fmaxf(z[r] + BD[kRHid + cD], 0.0f) + X0[rpad(cD)];
      }
    }
    __syncthreads();
    LZM_SUBSTAMP(33);
    int lrow = 0;  // the late draw's pick: the two-way tie's second candidate when rand() % 2 == 1
    if (NR == 1 && late) {
      const unsigned long long w0_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;
      if (G <= kRT) {
        // every wave looks back and draws for itself, so no barrier hands the pick over; wave 0 files it
        const int base = lookback_sum_w0(p, k, g, G, epoch);
        if (p.phase && tid == 0) s_wait += __builtin_amdgcn_s_memtime() - w0_;
        const uint32_t rr = glibc_draw_wave(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.diag);
        lrow = (int)(rr & 1u);  // (resolve_tie: rr % 2 over the mask's two set bits)
        if (tid == 0) resolve_tie(t, A, s_tlevel, s_tmask, rr, &s_act);
      } else {
        const int base = lookback_sum(p, k, g, G, epoch, s_part);
        if (p.phase && tid == 0) s_wait += __builtin_amdgcn_s_memtime() - w0_;
        if (tid == 0) resolve_tie(t, A, s_tlevel, s_tmask, glibc_draw(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.diag), &s_act);
        __syncthreads();
        lrow = s_act == act_r[1] ? 1 : 0;
      }
    }
    // the next latent row the rest of the network reads (NR = 1: the late draw's pick)
    const float *NLb = NL + ((NR == 1 && late && lrow) ? kRRow : 0);
    LZM_SUBSTAMP(34);
    LZM_STAMP(3);
    // The reward chain (fc_dynamics_2 -> reward head) and the prediction chain (prediction
    // common -> value / policy heads) both start from the next latent: one step per layer pair.
    // ---- [fc_dynamics_2[0] (LDS) | fc_prediction_common[0] (registers)]
    {
      float z2[NR], z6[NR];
      // fc_prediction_common[1] into P (used by the next pair), one slot per slot of this layer
      const __amdgpu_buffer_rsrc_t rd5 = wave_rsrc(res_blk4(n, kRbD + 5), kRSlotsD * kRT * 16);
      dense128n<NR>(NLb, [&](int j) { return WD2[j * kRT + tid]; }, z2, [&](int j) {
        const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rd5, tid * 16, j * kRT * 16, 0);
        P[j] = make_float4(v.x, v.y, v.z, v.w);
      });
      LZM_SUBSTAMP(35);
      dense128n<NR>(NLb, [&](int j) { return wD4[j]; }, z6);
      LZM_SUBSTAMP(36);
      if (pD == 0) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          T2[r * kRRow + rpad(cD)] = fmaxf(z2[r] + BD[2 * kRHid + cD], 0.0f);
          U2[r * kRRow + rpad(cD)] = fmaxf(z6[r] + BD[4 * kRHid + cD], 0.0f);
        }
      }
    }
    __syncthreads();
    LZM_SUBSTAMP(19);
    // ---- [fc_prediction_common[1] (streamed) | fc_dynamics_2[1] (registers)]
    {
      float z7[NR], z3[NR];
      dense128n<NR>(U2, [&](int j) { return P[j]; }, z7);
      LZM_SUBSTAMP(37);
      // the value support head into P (two steps on): half before this layer, half after it (a
      // 20-load burst stalls the wave at issue)
      __builtin_amdgcn_sched_barrier(0);
      const __amdgpu_buffer_rsrc_t rvs = wave_rsrc(res_blk4(n, kRbVS), kRSlotsS * kRT * 16);
      auto fetch_vs = [&](int q0, int q1) {
#pragma unroll
        for (int q = q0; q < q1; ++q) {
          const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rvs, tid * 16, q * kRT * 16, 0);
          P[q] = make_float4(v.x, v.y, v.z, v.w);
        }
      };
      fetch_vs(0, kRSlotsS / 2);
      dense128n<NR>(T2, [&](int j) { return wD3[j]; }, z3);
      LZM_SUBSTAMP(38);
      __builtin_amdgcn_sched_barrier(0);
      fetch_vs(kRSlotsS / 2, kRSlotsS);
      if (pD == 0) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          T3[r * kRRow + rpad(cD)] = fmaxf(z3[r] + BD[3 * kRHid + cD], 0.0f);
          U3[r * kRRow + rpad(cD)] = fmaxf(z7[r] + BD[5 * kRHid + cD], 0.0f);
        }
      }
    }
    __syncthreads();
    LZM_SUBSTAMP(39);
    LZM_STAMP(4);
    // ---- [reward head hidden | (value | policy) head hidden]
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      float h = dot4<kRSlotsRH>(reinterpret_cast<const float4 *>(T3 + r * kRRow) + 4 * pRH + (pRH >= 4),
                                [&](int j) { return wRH[j]; });
      float u = dot4<kRSlotsVPH>(reinterpret_cast<const float4 *>(U3 + r * kRRow) + 8 * pVP + (pVP >= 2),
                                 [&](int j) { return wVPH[j]; });
      h += dpp_f<0xB1>(h);
      u += dpp_f<0xB1>(u);
      h += dpp_f<0x4E>(h);
      u += dpp_f<0x4E>(u);
      h += dpp_f<0x141>(h);
      if (pRH == 0) RHo[r * kRF + cRH] = fmaxf(h + BRH[cRH], 0.0f);
      if (pVP == 0) HV[r * 2 * kRF + cVP] = fmaxf(u + BVP[cVP], 0.0f);
    }
    __syncthreads();
    LZM_STAMP(5);
    // ---- reward support (registers), value support (streamed), policy logits; every support
    // decoded together
    float dec[2 * NR];  // [row][reward, value]
    {
      float zz[2 * NR][3];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const float4 hp = reinterpret_cast<const float4 *>(HV + r * 2 * kRF + kRF)[tid & 7];
        float q = __fmaf_rn(hp.x, wPO[0].x, 0.0f);
        q = __fmaf_rn(hp.y, wPO[0].y, q);
        q = __fmaf_rn(hp.z, wPO[0].z, q);
        q = __fmaf_rn(hp.w, wPO[0].w, q);
        q += dpp_f<0xB1>(q);
        q += dpp_f<0x4E>(q);
        q += dpp_f<0x141>(q);
        if ((tid & 7) == 0 && cPO < A) LG[r * kRMaxA + cPO] = q + BPO[cPO];
        support_logits(HV + r * 2 * kRF, P, BVS, zz[2 * r + 1][0], zz[2 * r + 1][1], zz[2 * r + 1][2]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        support_logits(RHo + r * kRF, wRS, BRS, zz[2 * r][0], zz[2 * r][1], zz[2 * r][2]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      LZM_STAMP(15);
      support_decode_n<2 * NR>(zz, s_red, dec);
    }
    LZM_STAMP(6);
    // ---- resolve a speculative tie: the draw picks the row (predecessors published long ago)
    if (spec) {
      const int base = lookback_sum(p, k, g, G, epoch, s_part);
      if (tid == 0) resolve_tie(t, A, s_tlevel, s_tmask, glibc_draw(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.diag), &s_act);
      __syncthreads();
    }
    const int row = (spec && s_act == act_r[1]) ? 1 : 0;
    const float rdec = (NR == 2 && row) ? dec[2 * NR - 2] : dec[0];  // static indices: no scratch
    const float vdec = (NR == 2 && row) ? dec[2 * NR - 1] : dec[1];
    LZM_STAMP(7);
    if (p.phase && tid == 0) sub_ = __builtin_amdgcn_s_memtime();
    // file the next latent (mcts_ctree.py:305): pool[k + 1][i], by wave 1 (wave 0 expands)
    if (tid >= 64 && tid < 64 + kRHid / 4)
      reinterpret_cast<float4 *>(p.pool + ((size_t)(k + 1) * B + i) * kRHid)[tid - 64] =
          reinterpret_cast<const float4 *>(NLb + row * kRRow)[(tid - 64) + (tid - 64 >= kRHid / 8)];
    if (p.rec_x && tid == 0) {
      p.rec_x[(size_t)k * B + i] = s_x;
      p.rec_a[(size_t)k * B + i] = s_act;
      p.rec_len[(size_t)k * B + i] = s_len[0];
    }
    if (p.rec_dec && tid == 0) {
      p.rec_dec[((size_t)k * B + i) * 2] = rdec;
      p.rec_dec[((size_t)k * B + i) * 2 + 1] = vdec;
      for (int a = 0; a < A; ++a) p.rec_logits[((size_t)k * B + i) * A + a] = LG[row * kRMaxA + a];
    }
    // fc_dynamics[0] for the next simulation: wave 0 now, alone on the texture path (16 loads
    // issue in a few hundred cycles), waves 1-3 during the next walk, which only wave 0 runs
    LZM_SUBSTAMP(29);
    if (wid == 0) res_fetch<kRSlotsD>(res_blk4(n, kRbD), P);
    LZM_SUBSTAMP(30);
    // ---- expand + backup (cbatch_backpropagate, cnode.cpp:480-500): wave 0 files the leaf's own
    // record and backs up; wave 1 meanwhile initialises the leaf's children (disjoint nodes; the
    // next simulation's terms pass reads both after its barrier)
    if (wid == 0) {
      const int len = s_len[0];
      const int leaf = t.path[len];
      int vtp = s_vtp;
      if (players > 1)
        for (int l = 0; l < len; ++l) vtp = (vtp == 1) ? 2 : 1;
      LZM_SUBSTAMP(31);
      expand_wave(t, 0, leaf, vtp, k + 1, rdec, LG + row * kRMaxA, -1, s_exptab, 1);
      LZM_STAMP(14);
      if (lane == 0) L2N[s_nlat + k] = leaf;  // the leaf now holds latent k + 1 (= s_nlat + k)
      backup_wave(t, 0, 0, 1, &s_mm, vtp, vdec, p.disc);
    } else if (wid == 1) {
      expand_wave(t, 0, 0, 0, k + 1, 0.0f, LG + row * kRMaxA, -1, s_exptab, 2);
    }
    LZM_STAMP(9);
  }
  __syncthreads();
  LZM_STAMP(11);
  // ---- write back the slice (tree, min-max, last path)
  for (int e = tid; e < p.cap; e += kRT) {
    p.stat[(size_t)e * B + i] = t.stat[e];
    p.meta[(size_t)e * B + i] = t.meta[e];
  }
  for (int e = tid; e < p.depth_cap; e += kRT) {
    p.path[(size_t)e * B + i] = t.path[e];
    p.path_act[(size_t)e * B + i] = t.path_act[e];
  }
  if (tid == 0) {
    p.minmax[i] = s_mm;
    p.pathlen[i] = s_len[0];
  }
  // root outputs (root_outputs_kernel's values: visit counts per legal action, the root's value)
  if (p.out_dist && tid < A) {
    const int rl = t.meta[0].latent;
    p.out_dist[(size_t)i * A + tid] = (rl >= 0 && tid < t.nlegal[0]) ? t.stat[1 + A * rl + t.legal[tid]].visit : -1;
  }
  if (p.out_values && tid == 0) p.out_values[i] = node_value(t.stat[0]);
  __syncthreads();
  if (p.phase && tid < 64 && s_phase[tid]) atomicAdd(p.phase + tid, s_phase[tid]);
  if (p.phase && tid == 0 && g < 1024) atomicAdd(p.phase + 64 + g, s_wait);
  if (tid == 0) {
    // the last workgroup advances the epoch; no release fence (an L2 writeback per workgroup on
    // gfx950): the kernel boundary orders the write-back above for every later reader
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)G - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.step_count && p.step_inc) *p.step_count += 1;  // every workgroup has read it (its seeds)
    }
  }
}

}  // namespace lzm
