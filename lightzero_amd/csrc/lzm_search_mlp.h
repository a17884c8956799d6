// lzm_search_mlp.hip — one launch = one whole MuZero search (all simulations) for MLP models.
//
// Replaces, for the MuZeroModelMLP family (lzero/model/muzero_model_mlp.py:12-204), the whole
// per-simulation loop of MuZeroMCTSCtree.search (lzero/mcts/tree_search/mcts_ctree.py:255-321):
// traverse -> gather -> recurrent_inference -> InverseScalarTransform -> expand + backup.
//
// Decomposition. Workgroup g owns roots [g*R, g*R+R). Roots are independent trees, so a
// workgroup runs every simulation of its roots start to finish with its slice of the tree staged
// in LDS (node stats, search paths), the leaf latents gathered from the HBM pool
// [S+1][B][H], the network evaluated on its R rows (fp32 FMA; weights streamed from L2, each
// weight read once per workgroup per simulation), the reward/value supports decoded in LDS, the
// new latents filed into the pool, and the backup done in LDS. Nothing is exchanged between
// workgroups except, in parity mode, one 64-bit word per (simulation, workgroup): the number of
// rand() draws its roots consume, published for a decoupled look-back. The reference draws one
// rand() per tree level from a single stream in root order (cnode.cpp:592, :783), so root i's
// draws start at sum_{j<i} depth_j. A workgroup's depths almost never depend on the draws (a tie
// among unexpanded children ends the walk at the same depth whichever child wins), so it
// publishes its draw count at once, reads its predecessors' counts, and only then looks up the
// few draw values it needs — straight from the seeded state by a per-position coefficient table
// (random_r is linear over Z/2^32). Roots whose depth does depend on a draw are resolved after
// the predecessors' counts are known (exact serial semantics, slower). Fast mode uses Philox
// per (seed, root, level) and skips the look-back.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_numerics.h"
#include "lzm_tree.h"

namespace lzm {

#ifndef LZM_SEARCH_THREADS
#define LZM_SEARCH_THREADS 512
#endif
// Threads per search workgroup: two waves per SIMD. With fewer lanes the wide layers need more
// K-chunks per lane than the two-step prefetch holds in registers.
constexpr int kThreads = LZM_SEARCH_THREADS;


// One step of the network schedule, built on the host and read from the kernel arguments (scalar
// loads, no LDS round trips): the layer (kernel layout, see swz_source), its lane split, and the LDS
// float offsets of its input, output and residual.
struct StepRec {
  const float *w;  // lane-order weights, wbytes bytes
  const float *b;  // bias [N]
  int K, N, wbytes;  // K: inputs rounded up to kKC (zero rows)
  int in, out, relu, resid, rowmajor, ldout, decode;  // resid < 0: none; decode 1 reward, 2 value
  int Np, splits, cpl, log2s;                        // layer_split(K, N)
  // columns >= ncol1 (a second merged layer) read `in2` and store to `out2` (never decoded)
  int ncol1, in2, out2, rowmajor2, ldout2;
};

struct SearchArgs {
  // tree (HBM, whole batch)
  NodeStat *stat;
  NodeMeta *meta;
  const int32_t *legal, *nlegal;
  int32_t *path, *path_act, *pathlen;
  const float2 *lut;
  int B, A, cap, lut_n, depth_cap;
  // search
  int S;
  float disc;
  const uint32_t *seeds;  // [S]
  const int32_t *vtp_in;  // [B]
  float4 *minmax;         // [B]
  float *pool;            // [S+1][B][H]
  // network
  int H, F, V, res;
  // parity-mode draw table and look-back
  const uint32_t *coef;  // [P][31]
  int coef_positions;
  const uint32_t *pow16807;  // [31]
  unsigned long long *flags;  // [S][G]
  uint32_t *epoch;            // [2]: epoch, done counter
  int32_t *diag;              // [0] errors (spin timeouts), [1] ambiguous resolutions
  unsigned long long *phase;  // optional [16] per-phase shader-clock cycles (diagnostic builds)
  int fast;
  // optional per-simulation record (tests / tracing), may be null
  int32_t *rec_x, *rec_a, *rec_len;
  float *rec_dec, *rec_logits;
  // network schedule (host-built)
  StepRec sched[12];
  int nsteps, stamp_at[4];
  int diag_mode;  // timing experiments only (LZM_DIAG_MODE; results invalid): 1/3 weight loads out of range,
                  // 2 no dense FMAs, 4 no split-layer epilogue, 5 no step barrier, 6 no weight prefetch
  // dynamic LDS layout (float offsets)
  int tree_in_lds;
  size_t off_stat, off_meta, off_lut, off_legal, off_path, off_pact, off_x0, off_x1, off_x2, off_n, off_h, off_logit, off_part,
      off_misc, off_val, off_pbt;
  int pbt_rows;  // rows N of the pUCT visit table in LDS (0: none)
  // collect-step mode (lzm_search_set_step; the network-resident kernel runs it in-kernel):
  // step_count != null: seeds[k] = (step_base + *step_count * S + k) mod 10^6 instead of `seeds`,
  // and (step_inc) the last workgroup increments *step_count; mm_fresh: every root starts from fresh
  // min-max bounds (delta mm_delta); out_dist / out_values: the root outputs of
  // lzm_get_root_outputs, written by each root's workgroup after the search
  int64_t *step_count;
  int step_inc;  // the last workgroup increments *step_count
  long long step_base;
  int mm_fresh;
  float mm_delta;
  int32_t *out_dist;
  float *out_values;
};

// ------------------------------------------------------------------------------ LDS helpers
__device__ inline float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// Dense layers: out_T[n][r] (or out[r][n] when rowmajor) = act(in_T . W + b) (+ resid_T).
// A lane owns one output column for all R rows over a range of K; when a layer has fewer columns
// than lanes, `splits` lanes share a column (whole kKC-chunks each) and reduce through LDS.
// Each weight is read from L2 once per workgroup per simulation.
constexpr int kKC = 16;        // K-chunk: weights a lane holds in registers per group of FMAs
// Weight chunks per lane prefetched two schedule steps ahead into two register buffers: buffer A
// serves the even steps (including step 0, the widest: [latent; one-hot] rows), buffer B the odd
// ones. Wider R keeps fewer, its accumulators and input reads need the registers.
template <int R>
constexpr int pre_a() { return R == 1 ? 3 : (R == 2 ? 2 : 1); }
template <int R>
constexpr int pre_b() { return R == 1 ? 2 : 1; }
typedef const __attribute__((address_space(1))) float *gfloat_p;    // global (not flat) loads
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f32x4 *gfloat4_p;  // dwordx4 global loads

// Lane split of a layer with K inputs (K % kKC == 0) and N outputs, shared by the kernel and the
// host-side weight swizzle. splits == 0: wide layer (N >= kThreads), lane tid owns columns
// tid, tid + kThreads, ... over all K. Otherwise `splits` (a power of two <= 16) adjacent lanes
// share a column: lane = col * splits + part, col < Np (N rounded up to a power of two; columns
// >= N compute zeros), part p owns chunks [p * cpl, p * cpl + cpl) of K (chunks past K / kKC are
// skipped), and the partial sums meet through DPP lane exchanges, not LDS.
struct Split {
  int Np, splits, cpl, log2s;
};
__host__ __device__ inline Split layer_split(int K, int N) {
  Split s;
  const int nc = K / kKC;
  if (N >= kThreads) {
    s.Np = N; s.splits = 0; s.cpl = nc; s.log2s = 0;
    return s;
  }
  int Np = 1;
  while (Np < N) Np <<= 1;
  int sp = 1, lg = 0;
  while (sp < 16 && sp * 2 * Np <= kThreads && sp < nc) {
    sp *= 2;
    ++lg;
  }
  s.Np = Np; s.splits = sp; s.cpl = (nc + sp - 1) / sp; s.log2s = lg;
  return s;
}

// Kernel weight layout ("swizzled"): lane order, so that every wave-instruction of a layer's
// weight stream is one contiguous 1 KiB dwordx4 load. Split layer: float4 index
// (j * 4 + q) * (Np * splits) + lane holds W[k .. k+3][col], col = lane >> log2s,
// k = ((lane & (splits - 1)) * cpl + j) * kKC + 4q (zeros for col >= N or k >= K). Wide layer:
// round u (columns u * kThreads + lane, lane < n_u = min(kThreads, N - u * kThreads)) starts at
// float u * kThreads * K and holds float4 (j * 4 + q) * n_u + lane = W[j * kKC + 4q .. +3][col].
__host__ __device__ inline size_t swz_floats(int K, int N) {
  const Split s = layer_split(K, N);
  return s.splits ? (size_t)s.cpl * kKC * s.Np * s.splits : (size_t)K * N;
}
// Source (k, col) of kernel-layout float d of a layer; col >= N or k >= K marks padding.
__host__ __device__ inline void swz_source(int K, int N, size_t d, int *k, int *col) {
  const Split s = layer_split(K, N);
  const int e = (int)(d & 3);
  size_t f4 = d >> 2;
  if (s.splits) {
    const size_t nl = (size_t)s.Np * s.splits;
    const int lane = (int)(f4 % nl);
    const int q = (int)((f4 / nl) & 3);
    const int j = (int)(f4 / nl / 4);
    *col = lane >> s.log2s;
    *k = ((lane & (s.splits - 1)) * s.cpl + j) * kKC + 4 * q + e;
  } else {
    const size_t round = (size_t)kThreads * K;
    const int u = (int)(d / round);
    f4 = (d - (size_t)u * round) >> 2;
    const int nu = N - u * kThreads < kThreads ? N - u * kThreads : kThreads;
    const int lane = (int)(f4 % nu);
    const int q = (int)((f4 / nu) & 3);
    const int j = (int)(f4 / nu / 4);
    *col = u * kThreads + lane;
    *k = j * kKC + 4 * q + e;
  }
}


// chunk j of this lane: 4 float4 loads, lane stride nl (float4 units)
__device__ __forceinline__ void load_chunk(gfloat4_p base, int nl, int lane, int j, float *w) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 v = base[(size_t)(j * 4 + q) * nl + lane];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}

// Activations in LDS are transposed, [k][r], with a 4-float pad after every kKC rows of k: the
// lanes of a wave that split K read chunks a multiple of kKC apart, and the pad puts those reads
// on different banks.
template <int R>
__device__ __forceinline__ int tpos(int k, int r) { return (k / kKC) * (kKC * R + 4) + (k % kKC) * R + r; }

// acc[r] += sum_{j < kKC} inT[kb + j][r] * w[j] (R >= 2: k ascending, one fmaf per term). Inputs are
// broadcast LDS reads: one float4 covers 4 / R consecutive k for R < 4, or half a k for R = 8.
template <int R>
__device__ __forceinline__ void fma_chunk(const float *inT, int kb, const float *w, float *acc) {
  static_assert(R == 1 || R == 2 || R == 4 || R == 8, "rows per workgroup: 1, 2, 4 or 8");
  const float *cb = inT + tpos<R>(kb, 0);  // kb % kKC == 0: the chunk is contiguous
  if constexpr (R == 8) {
#pragma unroll
    for (int j = 0; j < kKC; ++j) {
      const float4 a0 = ld4(cb + j * R), a1 = ld4(cb + j * R + 4);
      acc[0] = __fmaf_rn(a0.x, w[j], acc[0]); acc[1] = __fmaf_rn(a0.y, w[j], acc[1]);
      acc[2] = __fmaf_rn(a0.z, w[j], acc[2]); acc[3] = __fmaf_rn(a0.w, w[j], acc[3]);
      acc[4] = __fmaf_rn(a1.x, w[j], acc[4]); acc[5] = __fmaf_rn(a1.y, w[j], acc[5]);
      acc[6] = __fmaf_rn(a1.z, w[j], acc[6]); acc[7] = __fmaf_rn(a1.w, w[j], acc[7]);
    }
  } else if constexpr (R == 4) {
#pragma unroll
    for (int j = 0; j < kKC; ++j) {
      const float4 a = ld4(cb + j * R);
      acc[0] = __fmaf_rn(a.x, w[j], acc[0]); acc[1] = __fmaf_rn(a.y, w[j], acc[1]);
      acc[2] = __fmaf_rn(a.z, w[j], acc[2]); acc[3] = __fmaf_rn(a.w, w[j], acc[3]);
    }
  } else if constexpr (R == 2) {
#pragma unroll
    for (int j = 0; j < kKC; j += 2) {
      const float4 a = ld4(cb + j * R);  // k = j: (x, y), k = j + 1: (z, w)
      acc[0] = __fmaf_rn(a.x, w[j], acc[0]); acc[1] = __fmaf_rn(a.y, w[j], acc[1]);
      acc[0] = __fmaf_rn(a.z, w[j + 1], acc[0]); acc[1] = __fmaf_rn(a.w, w[j + 1], acc[1]);
    }
  } else {
    // R = 1: four independent chains (k mod 4) instead of one 16-deep dependent chain
    float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < kKC; j += 4) {
      const float4 a = ld4(cb + j);
      a4[0] = __fmaf_rn(a.x, w[j], a4[0]); a4[1] = __fmaf_rn(a.y, w[j + 1], a4[1]);
      a4[2] = __fmaf_rn(a.z, w[j + 2], a4[2]); a4[3] = __fmaf_rn(a.w, w[j + 3], a4[3]);
    }
    acc[0] += (a4[0] + a4[1]) + (a4[2] + a4[3]);
  }
}

// Issue this lane's first kPreChunks weight chunks (and its bias) of a schedule step. Called right
// after the previous step's FMAs, so the L2 round trip overlaps that step's barrier, reduction and
// decode (and, for the first step of a simulation, the whole tree phase). Every register is
// (re)defined on every path, so no stale value stays live across the schedule loop.
// Buffer descriptor over `bytes` bytes at p, built from provably wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void *p, int bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kOOR = 0x7fffffff;  // out-of-range buffer offset: the load returns 0, no request

#ifndef LZM_PREFETCH_AHEAD
#define LZM_PREFETCH_AHEAD 2
#endif
// 1: each step prefetches the next step's weights, issuing exactly its chunk slots (uniform
//    branches; the compiler's conservative vmcnt at the consumer costs nothing one step ahead).
// 2: two register buffers, two steps ahead, branch-free fixed load counts (out-of-range slots).
constexpr int kPrefetchAhead = LZM_PREFETCH_AHEAD;

template <int kPreChunks>
__device__ __forceinline__ void prefetch_step(const StepRec &s, float *w, float &bias, bool diag_no_loads = false,
                                              bool diag_skip = false) {
  // Branch-free: every lane issues the same kPreChunks * 4 + 1 buffer loads; lanes (or chunks)
  // without data use an out-of-range offset, which returns zeros without a memory request. A fixed
  // load count per step lets s_waitcnt vmcnt wait for exactly the loads a step consumes while the
  // next step's stay in flight.
  const int tid = threadIdx.x;
  const int nl = s.splits ? s.Np * s.splits : (s.N < kThreads ? s.N : kThreads);
  const bool active = tid < nl;
  const int nc = s.K / kKC;
  const int c0 = s.splits ? (tid & (s.splits - 1)) * s.cpl : 0;
  const int n = active ? min(s.cpl, nc - c0) : 0;
  // the uniform part of each load's address lives in its descriptor (scalar ops); the lane part
  // is tid * 16, or out of range for lanes / chunk slots without data (one select per chunk)
  const char *wb = reinterpret_cast<const char *>(s.w);
  const int wbytes = diag_no_loads ? 0 : s.wbytes;
  // one-step-ahead: skip chunk slots no lane of the step has, and waves without any lane
  const bool wave_on = kPrefetchAhead == 1 ? (__builtin_amdgcn_readfirstlane(tid & ~63) < nl) : true;
#pragma unroll
  for (int c = 0; c < kPreChunks; ++c) {
    if (kPrefetchAhead == 1 && !(c < s.cpl && wave_on)) {
#pragma unroll
      for (int j = 0; j < kKC; ++j) w[c * kKC + j] = 0.0f;
      continue;
    }
    // (two-step-ahead) no branch around the loads, even for chunk slots no lane has: a branch makes
    // the load count path-dependent and the compiler then drains vmcnt conservatively
    const int vo = (c < n && !diag_skip) ? tid * 16 : kOOR;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int slot = (c * 4 + q) * nl * 16;  // byte offset of this (chunk, quarter) slot, uniform
      const int left = wbytes - slot;
      const __amdgpu_buffer_rsrc_t r = wave_rsrc(wb + slot, left > 0 ? left : 0);
      const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0);
      w[c * kKC + 4 * q] = v.x; w[c * kKC + 4 * q + 1] = v.y; w[c * kKC + 4 * q + 2] = v.z;
      w[c * kKC + 4 * q + 3] = v.w;
    }
  }
  const int col = s.splits ? tid >> s.log2s : tid;
  const bool lead = s.splits ? (tid & (s.splits - 1)) == 0 : true;  // adds the bias
  const __amdgpu_buffer_rsrc_t rb = wave_rsrc(s.b, s.N * 4);
  bias = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, (active && lead && col < s.N) ? col * 4 : kOOR, 0, 0));
}

// acc += chunks [j0, j1) of this lane streamed from L2, double-buffered.
template <int R>
__device__ __forceinline__ void dot_stream(gfloat4_p base, int nl, int lane, int j0, int j1, int kofs,
                                           const float *inT, float *acc) {
  float wa[kKC], wb[kKC];
  load_chunk(base, nl, lane, j0, wa);
  for (int j = j0; j < j1; j += 2) {
    const bool has_b = j + 1 < j1;
    if (has_b) load_chunk(base, nl, lane, j + 1, wb);
    fma_chunk<R>(inT, kofs + j * kKC, wa, acc);
    if (!has_b) break;
    if (j + 2 < j1) load_chunk(base, nl, lane, j + 2, wa);
    fma_chunk<R>(inT, kofs + (j + 1) * kKC, wb, acc);
  }
}

// acc += this lane's cnt chunks (k from kofs): the first pre_chunks from the prefetched w, the
// rest streamed.
template <int R, int kPreChunks>
__device__ __forceinline__ void dot_lane(gfloat4_p base, int nl, int lane, int cnt, int kofs, const float *inT,
                                         const float *w, float *acc) {
  if (cnt > 0) fma_chunk<R>(inT, kofs, w, acc);
  if (kPreChunks > 1 && cnt > 1) fma_chunk<R>(inT, kofs + kKC, w + kKC, acc);
  if (kPreChunks > 2 && cnt > 2) fma_chunk<R>(inT, kofs + 2 * kKC, w + 2 * kKC, acc);
  static_assert(kPreChunks >= 1 && kPreChunks <= 3, "prefetch depth");
  if (cnt > kPreChunks) dot_stream<R>(base, nl, lane, kPreChunks, cnt, kofs, inT, acc);
}


// Sum over each group of 2^log2s adjacent lanes (every lane of a group gets its group's sum):
// quad_perm xor 1, xor 2, then row_half_mirror and row_mirror pair the quads and half-rows.
template <int R>
__device__ __forceinline__ void group_sum(float *acc, int log2s) {
  if (log2s >= 1) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += dpp_f<0xB1>(acc[r]);
  }
  if (log2s >= 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += dpp_f<0x4E>(acc[r]);
  }
  if (log2s >= 3) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += dpp_f<0x141>(acc[r]);
  }
  if (log2s >= 4) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += dpp_f<0x140>(acc[r]);
  }
}

__device__ __forceinline__ float wave_max(float v) { return wave_max_dpp(v); }
// sum over the wave (rows of 16 by DPP, then the four row sums by readlane); every lane gets it
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}

constexpr int kWaves = kThreads / 64;
// column rounds of a wide layer whose support is decoded in registers (supports up to 1024)
constexpr int kMaxRounds = (1024 + kThreads - 1) / kThreads;

// out column c of a step: activation, residual, layout (columns >= ncol1: the second merged layer)
template <int R>
__device__ __forceinline__ void store_col(const StepRec &s, float *smem_f, const float *residT, int c, const float *v) {
  const bool second = c >= s.ncol1;
  float *out = smem_f + (second ? s.out2 : s.out);
  const int cc = second ? c - s.ncol1 : c;
  const int rowmajor = second ? s.rowmajor2 : s.rowmajor, ld = second ? s.ldout2 : s.ldout;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float x = v[r];
    if (s.relu) x = fmaxf(x, 0.0f);
    if (residT) x += residT[tpos<R>(c, r)];
    if (rowmajor) out[r * ld + cc] = x; else out[tpos<R>(cc, r)] = x;
  }
}

// One schedule step: out = act(in . W + b) (+ resid) for the workgroup's R rows, from the lane's
// prefetched weights `w`/`bias` (P chunks); right after its FMAs it issues the prefetch of step
// `sn` (two steps on) into the same registers. Wide layers with `decode` never store their logits: the categorical support
// expectation (scaling_transform.py:118-121: softmax, then sum p_j * (j - (V-1)/2)) is reduced
// across the workgroup from registers and h^-1 applied (InverseScalarTransform), into dec_out[r].
// `red`: 3 * kWaves * R floats of LDS. The caller's barrier follows.
template <int R, int P>
__device__ __forceinline__ void dense_step(const StepRec &s, float *smem_f, float *w, float &bias, float *red,
                                          float *dec_out, int nr, const StepRec &sn, int diag = 0) {
  const int tid = threadIdx.x;
  const int N = s.N;
  const float *residT = s.resid >= 0 ? smem_f + s.resid : nullptr;
  const bool wide = s.splits == 0;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = bias;
  float lg[kMaxRounds][R];  // wide + decode: logits of this lane's column rounds, static indices
  const int nl = wide ? kThreads : (s.Np << s.log2s);
  const int part = wide ? 0 : tid & (s.splits - 1), col = wide ? tid : tid >> s.log2s;
  // ---- FMAs (the prefetched registers are only read here)
  auto in_of = [&](int c) -> const float * { return smem_f + (c < s.ncol1 ? s.in : s.in2); };
  if (wide) {
    if (diag != 2) dot_lane<R, P>((gfloat4_p)s.w, kThreads, tid, s.cpl, 0, in_of(tid), w, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) lg[0][r] = acc[r];
    if (s.decode && tid >= s.ncol1) {  // a second-layer column already in round 0
      store_col<R>(s, smem_f, residT, tid, acc);
#pragma unroll
      for (int r = 0; r < R; ++r) lg[0][r] = -INFINITY;
    }
#pragma unroll
    for (int u = 1; u < kMaxRounds; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) lg[u][r] = -INFINITY;
      if (u * kThreads < N) {
        const int c = u * kThreads + tid;
        const int nu = N - u * kThreads < kThreads ? N - u * kThreads : kThreads;
        if (c < N) {
          float a2[R];
          const float b = ((gfloat_p)s.b)[c];
#pragma unroll
          for (int r = 0; r < R; ++r) a2[r] = b;
          dot_stream<R>((gfloat4_p)(s.w + (size_t)u * kThreads * s.K), nu, tid, 0, s.cpl, 0, in_of(c), a2);
          if (s.decode && c < s.ncol1) {
#pragma unroll
            for (int r = 0; r < R; ++r) lg[u][r] = a2[r];
          } else {
            store_col<R>(s, smem_f, residT, c, a2);
          }
        }
      }
    }
  } else {
    const int cnt = min(s.cpl, s.K / kKC - part * s.cpl);
    if (tid < nl && diag != 2) dot_lane<R, P>((gfloat4_p)s.w, nl, tid, cnt, part * s.cpl * kKC, in_of(col), w, acc);
  }
  // ---- the next-but-one step's weights: ONE definition point of the register buffer per step, so
  // the loop-carried registers need no copies at control-flow joins
  if (diag != 6) prefetch_step<P>(sn, w, bias, diag == 1, diag == 3);
  // ---- epilogue
  if (!wide) {
    if (tid < nl && diag != 4) {
      group_sum<R>(acc, s.log2s);
      if (part == 0 && col < N) store_col<R>(s, smem_f, residT, col, acc);
    }
    return;
  }
  if (!s.decode) {
    store_col<R>(s, smem_f, residT, tid, acc);
    return;
  }
  // fused support decode over the first ncol1 columns (<= kMaxRounds * kThreads, host-checked)
  const int wid = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float m = lg[0][r];
#pragma unroll
    for (int u = 1; u < kMaxRounds; ++u) m = fmaxf(m, lg[u][r]);
    m = wave_max(m);
    if (lane == 0) red[wid * R + r] = m;
  }
  __syncthreads();
  const int V = s.ncol1;
  const float half = (float)((V - 1) / 2);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float M = red[r];
    for (int q = 1; q < kWaves; ++q) M = fmaxf(M, red[q * R + r]);
    float se = 0.0f, sj = 0.0f;
#pragma unroll
    for (int u = 0; u < kMaxRounds; ++u) {
      if (u * kThreads + tid < N) {
        const float e = expf(lg[u][r] - M);
        se += e;
        sj += e * ((float)(u * kThreads + tid) - half);
      }
    }
    se = wave_sum(se);
    sj = wave_sum(sj);
    if (lane == 0) {
      red[(kWaves + wid) * R + r] = se;
      red[(2 * kWaves + wid) * R + r] = sj;
    }
  }
  __syncthreads();
  if (tid < nr) {
    float se = 0.0f, sj = 0.0f;
    for (int q = 0; q < kWaves; ++q) {
      se += red[(kWaves + q) * R + tid];
      sj += red[(2 * kWaves + q) * R + tid];
    }
    dec_out[tid] = h_inverse(sj / se);
  }
}

// Expectation of the categorical support of one row by one wave (scaling_transform.py:118-121).
__device__ inline float wave_expect_lds(const float *row, int V) {
  const int lane = threadIdx.x & 63;
  const float half = (float)((V - 1) / 2);
  float mx = -INFINITY;
  for (int j = lane; j < V; j += 64) mx = fmaxf(mx, row[j]);
  mx = xor_max(mx);
  float sum = 0.0f;
  for (int j = lane; j < V; j += 64) sum += expf(row[j] - mx);
  sum = xor_sum(sum);
  float acc = 0.0f;
  for (int j = lane; j < V; j += 64) acc += (expf(row[j] - mx) / sum) * ((float)j - half);
  acc = xor_sum(acc);
  return acc;
}

// glibc draw at absolute stream position p: (sum_j coef[p][j] * z0[j]) >> 1.
__device__ inline uint32_t glibc_draw(const uint32_t *coef, int positions, const uint32_t *z0, int p, int32_t *diag) {
  if (p >= positions) {
    atomicAdd(diag, 1);
    return 0u;
  }
  const uint32_t *c = coef + (size_t)p * 31;
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 31; ++j) v += c[j] * z0[j];
  return v >> 1;
}

// glibc_draw by a whole wave (p wave-uniform): lane j < 31 forms coefficient j's product and the wave adds
// them (mod 2^32, so in any order: the same value) — one round of loads and a butterfly instead of a
// 31-term dependent chain. Every lane returns the draw; all 64 lanes must call it.
__device__ __forceinline__ uint32_t glibc_draw_wave(const uint32_t *coef, int positions, const uint32_t *z0, int p,
                                                   int32_t *diag) {
  const int lane = threadIdx.x & 63;
  if (p >= positions) {
    if (lane == 0) atomicAdd(diag, 1);
    return 0u;
  }
  uint32_t v = lane < 31 ? coef[(size_t)p * 31 + lane] * z0[lane] : 0u;
  v += (uint32_t)xor_partner<32>((int)v);
  v += (uint32_t)xor_partner<16>((int)v);
  v += (uint32_t)xor_partner<8>((int)v);
  v += (uint32_t)xor_partner<4>((int)v);
  v += (uint32_t)xor_partner<2>((int)v);
  v += (uint32_t)xor_partner<1>((int)v);
  return v >> 1;
}

// The draws of one walk's levels lo .. lo + 63, one per lane (lane l: stream position
// base + lo + l), all coefficient rows in flight at once. cselect_child consumes a rand() at every
// level (cnode.cpp:587-590), so a walk resolved with draws paid one coefficient-row round trip per
// level through glibc_draw; through this it pays one. Built by a whole wave; operator() must be
// called wave-uniformly (readlane). Levels outside the window, or positions past the table, take
// glibc_draw (which flags the overflow) — the same values either way.
struct LaneDraws {
  const uint32_t *coef;
  const uint32_t *z0;
  int32_t *diag;
  int npos, base, lo;
  uint32_t v;
  __device__ uint32_t operator()(int level) const {
    const int l = level - lo;
    if (l >= 0 && l < 64 && base + level < npos) return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
    return glibc_draw(coef, npos, z0, base + level, diag);
  }
};
__device__ inline LaneDraws lane_draws(const uint32_t *coef, int npos, const uint32_t *z0, int base, int lo, int hi,
                                       int32_t *diag) {
  const int lane = threadIdx.x & 63;
  const int p = base + lo + lane;
  uint32_t v = 0;
  if (lo + lane < hi && p < npos) {
    const uint32_t *c = coef + (size_t)p * 31;
#pragma unroll
    for (int j = 0; j < 31; ++j) v += c[j] * z0[j];
    v >>= 1;
  }
  return LaneDraws{coef, z0, diag, npos, base, lo, v};
}

// z0[i] = seed * 16807^i mod (2^31 - 1) for seed in [1, 2^31-2] (srandom_r's Schrage loop
// computes exactly this); other seeds take the serial loop.
__device__ inline void seed_state_parallel(uint32_t seed, const uint32_t *pw, uint32_t *z0) {
  const int t = threadIdx.x;
  uint32_t s = seed == 0 ? 1u : seed;
  if (s < 0x7fffffffu) {
    if (t < 31) {
      unsigned long long x = (unsigned long long)s * pw[t];
      unsigned long long r = (x & 0x7fffffffull) + (x >> 31);
      r = (r & 0x7fffffffull) + (r >> 31);
      if (r >= 0x7fffffffull) r -= 0x7fffffffull;
      z0[t] = (uint32_t)r;
    }
  } else if (t == 0) {
    glibc_seed_state(seed, z0);
  }
}

// Phase stamps (diagnostics only; p.phase == nullptr in production): thread 0 of every
// workgroup adds the shader-clock cycles spent since the previous stamp to s_phase[n] (LDS), and
// flushes them into phase[] once at the end (no global atomics inside the timed phases).
#define LZM_STAMP(n)                                                              \
  do {                                                                            \
    if (p.phase && tid == 0) {                                                    \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();              \
      s_phase[n] += now_ - stamp_;                                                \
      stamp_ = now_;                                                              \
    }                                                                             \
  } while (0)

#define LZM_SUBSTAMP(n)                                                           \
  do {                                                                            \
    if (p.phase && tid == 0) {                                                    \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();              \
      s_phase[n] += now_ - sub_;                                                  \
      sub_ = now_;                                                                \
    }                                                                             \
  } while (0)

// TL: the workgroup's tree slice (node records, pUCT table, root legal lists) is staged in LDS
// for the whole search; otherwise the nodes stay in HBM (large action spaces x simulations).
// The pUCT visit table lpbt[n (n + 1) / 2 + v] = lut[n].y / (v + 1) for v <= n < rows, one entry
// per thread: every lut load is independent (one memory round trip, not one per row).
__device__ inline void build_pbt(const float2 *lut, int rows, float *lpbt, int tid, int nthreads) {
  const int total = rows * (rows + 1) / 2;
  for (int e = tid; e < total; e += nthreads) {
    int n = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    while (n > 0 && n * (n + 1) / 2 > e) --n;
    while ((n + 1) * (n + 2) / 2 <= e) ++n;
    const int v = e - n * (n + 1) / 2;
    lpbt[e] = lut[n].y / (float)(v + 1);
  }
}

template <int R, bool TL>
__global__ __launch_bounds__(kThreads) void search_mlp_kernel(SearchArgs p) {
  extern __shared__ float4 smem4[];
  float *smem = reinterpret_cast<float *>(smem4);
  const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x;
  const int B = p.B, A = p.A, H = p.H;
  const int i0 = g * R;
  const int nr = min(R, B - i0);  // roots in this slice
  unsigned long long stamp_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;

  __shared__ uint32_t s_z0[31];
  __shared__ int s_players, s_base, s_flag, s_epoch;
  __shared__ int s_x[R], s_act[R], s_len[R], s_status[R], s_tlevel[R], s_off[R], s_vtp[R];
  __shared__ unsigned long long s_tmask[R];
  __shared__ float s_r[R], s_v[R];
  __shared__ float4 s_mm[R];
  __shared__ unsigned long long s_phase[64];
  __shared__ float s_red[3 * kWaves * R];
  if (p.phase && tid < 64) s_phase[tid] = 0ull;

  // ---- stage the tree slice and per-root state
  TreeView t;
  t.A = A;
  t.cap = p.cap;
  t.lut_n = p.lut_n;
  t.depth_cap = p.depth_cap;
  t.path = reinterpret_cast<int32_t *>(smem + p.off_path);
  t.path_act = reinterpret_cast<int32_t *>(smem + p.off_pact);
  t.pathlen = s_len;
  if constexpr (TL) {
    NodeStat *ls = reinterpret_cast<NodeStat *>(smem + p.off_stat);
    NodeMeta *lm = reinterpret_cast<NodeMeta *>(smem + p.off_meta);
    float2 *llut = reinterpret_cast<float2 *>(smem + p.off_lut);
    int32_t *llegal = reinterpret_cast<int32_t *>(smem + p.off_legal);
    for (int e = tid; e < p.cap * R; e += kThreads) {
      const int node = e / R, li = e % R;
      if (li < nr) {
        ls[e] = p.stat[(size_t)node * B + i0 + li];
        lm[e] = p.meta[(size_t)node * B + i0 + li];
      }
    }
    for (int e = tid; e < p.lut_n; e += kThreads) llut[e] = p.lut[e];
    // caches replacing the descent's divisions (bit-identical: same operands, same IEEE division)
    float *lval = smem + p.off_val;
    for (int e = tid; e < p.cap * R; e += kThreads) {
      const int node = e / R, li = e % R;
      lval[e] = li < nr ? node_value(p.stat[(size_t)node * B + i0 + li]) : 0.0f;
    }
    float *lpbt = smem + p.off_pbt;
    build_pbt(p.lut, p.pbt_rows, lpbt, tid, kThreads);
    t.val = lval;
    t.pbt = p.pbt_rows ? lpbt : nullptr;
    for (int e = tid; e < R * A; e += kThreads) llegal[e] = (e / A < nr) ? p.legal[(size_t)i0 * A + e] : 0;
    for (int e = tid; e < R; e += kThreads) llegal[R * A + e] = (e < nr) ? p.nlegal[i0 + e] : 0;
    t.stat = ls;
    t.meta = lm;
    t.lut = llut;
    t.legal = llegal;
    t.nlegal = llegal + R * A;
    t.B = R;
  } else {
    t.stat = p.stat;
    t.meta = p.meta;
    t.lut = p.lut;
    t.legal = p.legal;
    t.nlegal = p.nlegal;
    t.B = B;
  }
  // tree index of local root li: li in the LDS slice, i0 + li in the HBM batch
  auto tix = [i0](int li) { return TL ? li : i0 + li; };
  if (tid < R && tid < nr) {
    s_mm[tid] = p.minmax[i0 + tid];
    s_vtp[tid] = p.vtp_in[i0 + tid];
  }
  if (tid == 0) s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < 64) {
    // players (cnode.cpp:776-781) by wave 0, every load in flight at once
    int m = INT_MIN;
    for (int q = tid; q < B; q += 64) m = max(m, p.vtp_in[q]);
    m = xor_max(m);
    if (tid == 0) s_players = (m == -1) ? 1 : 2;
  }
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;

  uint32_t *s_seeds = reinterpret_cast<uint32_t *>(smem + p.off_misc);
  uint32_t *s_pow = s_seeds + p.S;
  for (int e = tid; e < p.S; e += kThreads) s_seeds[e] = p.seeds[e];
  if (!p.fast)
    for (int e = tid; e < 31; e += kThreads) s_pow[e] = p.pow16807[e];
  __syncthreads();
  LZM_STAMP(10);
  float *X0 = smem + p.off_x0, *X1 = smem + p.off_x1, *NL = smem + p.off_n;
  float *LG = smem + p.off_logit;
  // this lane's weights for the next schedule step, loaded one step ahead (prefetch_step)
  // weight prefetch buffers: two-step-ahead: A for even schedule steps, B for odd (schedules have an
  // even length); one-step-ahead: A only
  float wA[pre_a<R>() * kKC], bA = 0.0f, wB[pre_b<R>() * kKC], bB = 0.0f;
  prefetch_step<pre_a<R>()>(p.sched[0], wA, bA);
  if (kPrefetchAhead == 2) prefetch_step<pre_b<R>()>(p.sched[1], wB, bB);

  for (int k = 0; k < p.S; ++k) {
    const uint32_t seed = s_seeds[k];
    if (!p.fast) seed_state_parallel(seed, s_pow, s_z0);
    // ---- selection: wave w walks roots w, w + kWaves, ... (one lane per child, descend_wave)
    for (int li = tid >> 6; li < nr; li += kWaves) {
      const int i = i0 + li;
      const TreeView &tv = t;
      const int ti = tix(li);
      const bool lead = (tid & 63) == 0;
      if (p.fast) {
        auto draw = [seed, i](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)i, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        Descent d = descend_wave<false, false>(tv, ti, li, R, s_mm[li], players, s_vtp[li], p.disc, draw, nullptr);
        if (lead) { s_len[li] = d.len; s_x[li] = d.x; s_act[li] = d.action; s_status[li] = 0; }
      } else {
        // classification pass: no draw values needed unless a tie involves an expanded child
        TieInfo ti_info;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        Descent d = descend_wave<false, true>(tv, ti, li, R, s_mm[li], players, s_vtp[li], p.disc, nodraw, &ti_info);
        if (lead) {
          s_len[li] = d.len; s_x[li] = d.x; s_act[li] = d.action;
          s_status[li] = ti_info.status;
          s_tlevel[li] = ti_info.level;
          s_tmask[li] = ti_info.mask;
        }
      }
    }
    __syncthreads();
    LZM_STAMP(0);
    if (!p.fast) {
      // ---- draw offsets: publish this slice's draw count, look back over predecessors
      if (tid == 0) {
        int ambiguous = 0, total = 0;
        for (int li = 0; li < nr; ++li) {
          s_off[li] = total;
          total += s_len[li];
          ambiguous |= (s_status[li] == 2);
        }
        s_flag = ambiguous;
        if (!ambiguous)
          __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)total, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      // base = sum of predecessors' draw counts (wave 0 polls; bounded spin)
      if (tid < 64) {
        int sum = 0;
        for (int q = tid; q < g; q += 64) {
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
        if (tid == 0) s_base = sum;
      }
      __syncthreads();
      const int base = s_base;
      if (s_flag) {
        // some root's depth depends on its draws: resolve the slice serially (exact semantics)
        if (tid == 0) {
          atomicAdd(p.diag + 1, 1);
          int total = 0;
          for (int li = 0; li < nr; ++li) {
            const TreeView &tv = t;
            const int ti = tix(li);
            const int off = base + total;
            const uint32_t *coef = p.coef;
            const int npos = p.coef_positions;
            int32_t *diag = p.diag;
            auto draw = [coef, npos, diag, off](int level) -> uint32_t {
              return glibc_draw(coef, npos, s_z0, off + level, diag);
            };
            Descent d = descend_slice<false, false>(tv, ti, li, R, s_mm[li], players, s_vtp[li], p.disc, draw, nullptr);
            s_len[li] = d.len; s_x[li] = d.x; s_act[li] = d.action; s_status[li] = 0;
            total += d.len;
          }
          __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)total, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      } else if (tid < nr) {
        // resolve the one pending tie (if any) of each root with its draw
        const int li = tid;
        if (s_status[li] == 1) {
          const uint32_t rr = glibc_draw(p.coef, p.coef_positions, s_z0, base + s_off[li] + s_tlevel[li], p.diag);
          unsigned long long m = s_tmask[li];
          int kk = (int)(rr % (uint32_t)__popcll(m));
          for (; kk > 0; --kk) m &= m - 1;
          const int jsel = __ffsll((long long)m) - 1;
          const TreeView &tv = t;
          const int ti = tix(li);
          const int lvl = s_tlevel[li];
          const int parent = tv.path[lvl * R + li];
          const int action = legal_at(tv, ti, parent, jsel);
          const int base_child = 1 + A * tv.meta[nidx(tv, parent, ti)].latent;
          tv.path_act[lvl * R + li] = action;
          tv.path[(lvl + 1) * R + li] = base_child + action;
          s_act[li] = action;
          s_x[li] = tv.meta[nidx(tv, parent, ti)].latent;
        }
      }
      __syncthreads();
    }
    if (p.rec_x && tid < nr) {
      p.rec_x[(size_t)k * B + i0 + tid] = s_x[tid];
      p.rec_a[(size_t)k * B + i0 + tid] = s_act[tid];
      p.rec_len[(size_t)k * B + i0 + tid] = s_len[tid];
    }
    LZM_STAMP(1);
    // ---- gather leaf latents: X0[h][r] = pool[x_r][i0+r][h]
    for (int e = tid; e < H * R; e += kThreads) {
      const int r = e / H, h = e % H;
      float v = 0.0f;
      if (r < nr) v = p.pool[((size_t)max(s_x[r], 0) * B + i0 + r) * H + h];
      X0[tpos<R>(h, r)] = v;
    }
    // one-hot action rows H .. K0 (layer 0's zero-padded input; muzero_model_mlp.py:188-190)
    for (int e = tid; e < (p.sched[0].K - H) * R; e += kThreads) {
      const int a = e / R, r = e % R;
      X0[tpos<R>(H + a, r)] = (r < nr && s_act[r] == a) ? 1.0f : 0.0f;
    }
    __syncthreads();
    LZM_STAMP(2);
    // ---- network (recurrent_inference, BN folded): muzero_model_mlp.py:179-204, :420-440
    // The schedule (p.sched) walks: fc_dynamics(_1) (+ one-hot action,
    // + residual), fc_dynamics_2, reward head (-> decode into s_r), fc_prediction_common, value
    // head (-> decode into s_v), policy head (-> logits [r][A] in X1).
    // schedule, unrolled by two so each register buffer has a fixed place in the instruction
    // stream: even steps consume buffer A, odd steps B; each refills its buffer for two steps on
    // (wrapping into the next simulation's first two steps)
#define LZM_NET_STEP(ST, W, BIAS, P)                                                                  \
  do {                                                                                               \
    const int st_ = (ST);                                                                            \
    const StepRec &q = p.sched[st_];                                                                 \
    unsigned long long sub_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;                         \
    const int nx = st_ + kPrefetchAhead < p.nsteps ? st_ + kPrefetchAhead : st_ + kPrefetchAhead - p.nsteps; \
    float *dec = q.decode == 1 ? s_r : s_v;                                                          \
    dense_step<R, P>(q, smem, W, BIAS, s_red, dec, nr, p.sched[nx], p.diag_mode);                    \
    LZM_SUBSTAMP(16 + 4 * st_);                                                                      \
    if (p.diag_mode != 5) __syncthreads();                                                           \
    LZM_SUBSTAMP(17 + 4 * st_);                                                                      \
    if (q.decode && q.splits) { /* narrow support (< kThreads): logits in LG, one wave per row */    \
      for (int r = tid >> 6; r < nr; r += kWaves) {                                                  \
        const float e = wave_expect_lds(LG + r * (p.V + 1), p.V);                                    \
        if ((tid & 63) == 0) dec[r] = h_inverse(e);                                                  \
      }                                                                                              \
      __syncthreads();                                                                               \
    }                                                                                                \
    if (st_ == p.stamp_at[0]) LZM_STAMP(3);                                                          \
    if (st_ == p.stamp_at[1]) LZM_STAMP(4);                                                          \
    if (st_ == p.stamp_at[2]) LZM_STAMP(5);                                                          \
    if (st_ == p.stamp_at[3]) LZM_STAMP(6);                                                          \
  } while (0)
    if (kPrefetchAhead == 2) {
      for (int st = 0; st < p.nsteps; st += 2) {
        LZM_NET_STEP(st, wA, bA, pre_a<R>());
        LZM_NET_STEP(st + 1, wB, bB, pre_b<R>());
      }
    } else {
      for (int st = 0; st < p.nsteps; ++st) LZM_NET_STEP(st, wA, bA, pre_a<R>());
    }
#undef LZM_NET_STEP
    LZM_STAMP(7);
    // ---- file the new latents (mcts_ctree.py:305): pool[k+1][i][h] = NL[h][r]
    for (int e = tid; e < H * R; e += kThreads) {
      const int r = e / H, h = e % H;
      if (r < nr) p.pool[((size_t)(k + 1) * B + i0 + r) * H + h] = NL[tpos<R>(h, r)];
    }
    if (p.rec_dec && tid < nr) {
      p.rec_dec[((size_t)k * B + i0 + tid) * 2] = s_r[tid];
      p.rec_dec[((size_t)k * B + i0 + tid) * 2 + 1] = s_v[tid];
      for (int a = 0; a < A; ++a) p.rec_logits[((size_t)k * B + i0 + tid) * A + a] = X1[tid * A + a];
    }
    LZM_STAMP(8);
    // ---- expand + backup (cbatch_backpropagate, cnode.cpp:480-500): wave w takes root w, one lane
    // per child (expand) and per path level (backup)
    for (int li = tid >> 6; li < nr; li += kWaves) {
      const TreeView &tv = t;
      const int ti = tix(li);
      const int len = s_len[li];
      const int leaf = tv.path[len * R + li];
      int vtp = s_vtp[li];
      if (players > 1)
        for (int l = 0; l < len; ++l) vtp = (vtp == 1) ? 2 : 1;
      expand_wave(tv, ti, leaf, vtp, k + 1, s_r[li], X1 + li * A);
      backup_wave(tv, ti, li, R, &s_mm[li], vtp, s_v[li], p.disc);
    }
    __syncthreads();
    LZM_STAMP(9);
  }
  // ---- write back the slice (tree, min-max, last paths)
  LZM_STAMP(11);
  if constexpr (TL) {
    for (int e = tid; e < p.cap * R; e += kThreads) {
      const int node = e / R, li = e % R;
      if (li < nr) {
        p.stat[(size_t)node * B + i0 + li] = t.stat[e];
        p.meta[(size_t)node * B + i0 + li] = t.meta[e];
      }
    }
  }
  for (int e = tid; e < p.depth_cap * R; e += kThreads) {
    const int l = e / R, li = e % R;
    if (li < nr) {
      p.path[(size_t)l * B + i0 + li] = t.path[e];
      p.path_act[(size_t)l * B + i0 + li] = t.path_act[e];
    }
  }
  if (tid < nr) {
    p.minmax[i0 + tid] = s_mm[tid];
    p.pathlen[i0 + tid] = s_len[tid];
  }
  // epoch advance by the last workgroup to finish (the next launch reads the new epoch)
  __syncthreads();
  if (p.phase && tid < 64 && s_phase[tid]) atomicAdd(p.phase + tid, s_phase[tid]);
  if (tid == 0) {
    // the last workgroup advances the epoch; no release fence (an L2 writeback per workgroup on
    // gfx950): the kernel boundary orders the write-back above for every later reader
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)G - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace lzm
