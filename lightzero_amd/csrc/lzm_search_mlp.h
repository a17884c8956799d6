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

constexpr int kThreads = 512;  // 8 waves: two per SIMD, so one's memory wait hides under the other's FMAs

struct MlpLayer {
  const float *w;  // [K][ldw] (input-major), zero-padded columns
  const float *b;  // [ldw]
  int K, N, ldw;
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
  MlpLayer L[12];
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
  // dynamic LDS layout (float offsets)
  int tree_in_lds;
  size_t off_stat, off_meta, off_lut, off_legal, off_path, off_pact, off_x0, off_x1, off_x2, off_n, off_h, off_logit, off_part,
      off_misc;
};

// ------------------------------------------------------------------------------ LDS helpers
__device__ inline float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// out_T[n][r] (or out[r][n] when rowmajor) = act(in_T . W + b (+ W[H+a_r] one-hot row)) (+ resid_T)
// Each weight element is read from L2 by exactly one lane: a lane owns one output column for all
// R rows; spare lanes split K and reduce through LDS partials.
constexpr int kKC = 16;  // weights held in registers per lane before the FMAs that use them
typedef const __attribute__((address_space(1))) float *gfloat_p;  // global (not flat) loads

// acc[r] += sum_{k in [k0, k1)} inT[k][r] * W[k][col] with (k1 - k0) % kKC == 0: each chunk's
// weights are issued as loads first, so one L2 round trip is paid per chunk, not per weight.
template <int R>
__device__ __forceinline__ void load_chunk(gfloat_p W, int ldw, int col, int kb, float *w) {
#pragma unroll
  for (int j = 0; j < kKC; ++j) w[j] = W[(size_t)(kb + j) * ldw + col];
}

template <int R>
__device__ __forceinline__ void fma_chunk(const float *inT, int kb, const float *w, float *acc) {
#pragma unroll
  for (int j = 0; j < kKC; ++j) {
    const float4 a0 = ld4(inT + (kb + j) * R), a1 = ld4(inT + (kb + j) * R + 4);
    acc[0] = __fmaf_rn(a0.x, w[j], acc[0]); acc[1] = __fmaf_rn(a0.y, w[j], acc[1]);
    acc[2] = __fmaf_rn(a0.z, w[j], acc[2]); acc[3] = __fmaf_rn(a0.w, w[j], acc[3]);
    acc[4] = __fmaf_rn(a1.x, w[j], acc[4]); acc[5] = __fmaf_rn(a1.y, w[j], acc[5]);
    acc[6] = __fmaf_rn(a1.z, w[j], acc[6]); acc[7] = __fmaf_rn(a1.w, w[j], acc[7]);
  }
}

// Double-buffered: the next chunk's weight loads are in flight while this chunk's FMAs issue.
template <int R>
__device__ __forceinline__ void dot_chunked(gfloat_p W, int ldw, int col, int k0, int k1, const float *inT,
                                            float *acc) {
  float wa[kKC], wb[kKC];
  load_chunk<R>(W, ldw, col, k0, wa);
  for (int kb = k0; kb < k1; kb += 2 * kKC) {
    const bool has_b = kb + kKC < k1;
    if (has_b) load_chunk<R>(W, ldw, col, kb + kKC, wb);
    fma_chunk<R>(inT, kb, wa, acc);
    if (!has_b) break;
    if (kb + 2 * kKC < k1) load_chunk<R>(W, ldw, col, kb + 2 * kKC, wa);
    fma_chunk<R>(inT, kb + kKC, wb, acc);
  }
}

// One network layer on the workgroup's R rows (K % kKC == 0, checked on the host). Called from a
// loop over the layer schedule, so its code exists once (the loop body must fit the I-cache).
template <int R>
__device__ __forceinline__ void dense(const MlpLayer L, const float *inT, float *out, float *part, int relu,
                                   const float *residT, int rowmajor, int ldout, const int *onehot_act,
                                   int onehot_row0) {
  static_assert(R == 8, "dense is written for 8 rows per workgroup");
  const int tid = threadIdx.x;
  const int N = L.N, K = L.K;
  gfloat_p W = (gfloat_p)L.w;
  gfloat_p Bv = (gfloat_p)L.b;
  if (N >= kThreads) {
    for (int c = tid; c < N; c += kThreads) {
      float acc[R];
      const float bias = Bv[c];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = bias;
      dot_chunked<R>(W, L.ldw, c, 0, K, inT, acc);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float v = acc[r];
        if (relu) v = fmaxf(v, 0.0f);
        if (rowmajor) out[r * ldout + c] = v; else out[c * R + r] = v;
      }
    }
    __syncthreads();
    return;
  }
  // split K over up to kThreads / Np lanes per column, whole chunks per lane
  int Np = 1;
  while (Np < N) Np <<= 1;
  int splits = min(kThreads / Np, K / kKC);
  while ((K / kKC) % splits) --splits;  // whole chunks per lane
  const int col = tid % Np, part_id = tid / Np;
  const int kchunk = K / splits;  // multiple of kKC
  float acc[R];
  const bool active = col < N && part_id < splits;
  const float bias = (active && part_id == 0) ? Bv[col] : 0.0f;
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = bias;
  if (active) {
    if (onehot_act && part_id == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] += W[(size_t)(onehot_row0 + onehot_act[r]) * L.ldw + col];
    }
    dot_chunked<R>(W, L.ldw, col, part_id * kchunk, part_id * kchunk + kchunk, inT, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) part[(part_id * Np + col) * R + r] = acc[r];
  }
  __syncthreads();
  for (int e = tid; e < N * R; e += kThreads) {
    const int c = e / R, r = e % R;
    float v = part[c * R + r];
    for (int s = 1; s < splits; ++s) v += part[(s * Np + c) * R + r];
    if (relu) v = fmaxf(v, 0.0f);
    if (residT) v += residT[c * R + r];
    if (rowmajor) out[r * ldout + c] = v; else out[c * R + r] = v;
  }
  __syncthreads();
}

// Expectation of the categorical support of one row by one wave (scaling_transform.py:118-121).
__device__ inline float wave_expect_lds(const float *row, int V) {
  const int lane = threadIdx.x & 63;
  const float half = (float)((V - 1) / 2);
  float mx = -INFINITY;
  for (int j = lane; j < V; j += 64) mx = fmaxf(mx, row[j]);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = fmaxf(mx, __shfl_xor(mx, d, 64));
  float sum = 0.0f;
  for (int j = lane; j < V; j += 64) sum += expf(row[j] - mx);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
  float acc = 0.0f;
  for (int j = lane; j < V; j += 64) acc += (expf(row[j] - mx) / sum) * ((float)j - half);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
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
// workgroup adds the shader-clock cycles spent since the previous stamp to phase[n].
#define LZM_STAMP(n)                                                              \
  do {                                                                            \
    if (p.phase && tid == 0) {                                                    \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();              \
      atomicAdd(p.phase + (n), now_ - stamp_);                                   \
      stamp_ = now_;                                                              \
    }                                                                             \
  } while (0)

// TL: the workgroup's tree slice (node records, pUCT table, root legal lists) is staged in LDS
// for the whole search; otherwise the nodes stay in HBM (large action spaces x simulations).
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
  __shared__ MlpLayer s_L[12];
  __shared__ int s_step[12][9];
  __shared__ int s_nsteps, s_stamp_at[4];

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
  if (tid == 0) {
    int m = INT_MIN;
    for (int i = 0; i < B; ++i) m = max(m, p.vtp_in[i]);
    s_players = (m == -1) ? 1 : 2;
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int l = 0; l < 12; ++l) s_L[l] = p.L[l];
    // layer schedule: {layer, in, out, relu, resid (-1: none), rowmajor, ldout, one-hot, decode}
    const int x0 = (int)p.off_x0, x1 = (int)p.off_x1, x2 = (int)p.off_x2, nl = (int)p.off_n, hd = (int)p.off_h,
              lg = (int)p.off_logit;
    int n = 0;
    auto add = [&](int l, int in, int out, int relu, int resid, int rowmajor, int ldout, int onehot, int dec) {
      int *q = s_step[n++];
      q[0] = l; q[1] = in; q[2] = out; q[3] = relu; q[4] = resid; q[5] = rowmajor; q[6] = ldout; q[7] = onehot;
      q[8] = dec;
    };
    add(0, x0, x1, 1, -1, 0, 0, 1, 0);                   // fc_dynamics(_1)[0] on [latent; one-hot]
    add(1, x1, nl, 1, p.res ? x0 : -1, 0, 0, 0, 0);      // [1] (+ latent: res_connection_in_dynamics)
    int enc = nl;
    if (p.res) {
      add(2, nl, x1, 1, -1, 0, 0, 0, 0);                 // fc_dynamics_2
      add(3, x1, x2, 1, -1, 0, 0, 0, 0);
      enc = x2;
    }
    s_stamp_at[0] = n - 1;
    add(4, enc, hd, 1, -1, 0, 0, 0, 0);                  // fc_reward_head
    add(5, hd, lg, 0, -1, 1, p.V + 1, 0, 1);
    s_stamp_at[1] = n - 1;
    add(6, nl, x1, 1, -1, 0, 0, 0, 0);                   // fc_prediction_common
    add(7, x1, x2, 1, -1, 0, 0, 0, 0);
    s_stamp_at[2] = n - 1;
    add(8, x2, hd, 1, -1, 0, 0, 0, 0);                   // fc_value_head
    add(9, hd, lg, 0, -1, 1, p.V + 1, 0, 2);
    s_stamp_at[3] = n - 1;
    add(10, x2, hd, 1, -1, 0, 0, 0, 0);                  // fc_policy_head
    add(11, hd, x1, 0, -1, 1, A, 0, 0);
    s_nsteps = n;
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
  float *X0 = smem + p.off_x0, *X1 = smem + p.off_x1, *X2 = smem + p.off_x2, *NL = smem + p.off_n;
  float *HD = smem + p.off_h, *LG = smem + p.off_logit, *PART = smem + p.off_part;

  for (int k = 0; k < p.S; ++k) {
    const uint32_t seed = s_seeds[k];
    if (!p.fast) seed_state_parallel(seed, s_pow, s_z0);
    // ---- selection
    if (tid < nr) {
      const int li = tid, i = i0 + li;
      const TreeView &tv = t;
      const int ti = tix(li);
      if (p.fast) {
        auto draw = [seed, i](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)i, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        Descent d = descend_slice<false, false>(tv, ti, li, R, s_mm[li], players, s_vtp[li], p.disc, draw, nullptr);
        s_len[li] = d.len; s_x[li] = d.x; s_act[li] = d.action; s_status[li] = 0;
      } else {
        // classification pass: no draw values needed unless a tie involves an expanded child
        TieInfo ti_info;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        Descent d = descend_slice<false, true>(tv, ti, li, R, s_mm[li], players, s_vtp[li], p.disc, nodraw, &ti_info);
        s_len[li] = d.len; s_x[li] = d.x; s_act[li] = d.action;
        s_status[li] = ti_info.status;
        s_tlevel[li] = ti_info.level;
        s_tmask[li] = ti_info.mask;
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
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
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
      X0[h * R + r] = v;
    }
    __syncthreads();
    LZM_STAMP(2);
    // ---- network (recurrent_inference, BN folded): muzero_model_mlp.py:179-204, :420-440
    // One dense() instance walks the layer schedule (s_step): fc_dynamics(_1) (+ one-hot action,
    // + residual), fc_dynamics_2, reward head (-> decode into s_r), fc_prediction_common, value
    // head (-> decode into s_v), policy head (-> logits [r][A] in X1).
    for (int st = 0; st < s_nsteps; ++st) {
      const int *q = s_step[st];
      dense<R>(s_L[q[0]], smem + q[1], smem + q[2], PART, q[3], q[4] >= 0 ? smem + q[4] : nullptr, q[5], q[6],
               q[7] ? s_act : nullptr, H);
      if (q[8]) {  // decode the support logits just produced (InverseScalarTransform)
        const int wid = tid >> 6;
        for (int r = wid; r < nr; r += kThreads / 64) {
          const float e = wave_expect_lds(LG + r * (p.V + 1), p.V);
          if ((tid & 63) == 0) (q[8] == 1 ? s_r : s_v)[r] = h_inverse(e);
        }
        __syncthreads();
      }
      if (st == s_stamp_at[0]) LZM_STAMP(3);
      if (st == s_stamp_at[1]) LZM_STAMP(4);
      if (st == s_stamp_at[2]) LZM_STAMP(5);
      if (st == s_stamp_at[3]) LZM_STAMP(6);
    }
    LZM_STAMP(7);
    // ---- file the new latents (mcts_ctree.py:305): pool[k+1][i][h] = NL[h][r]
    for (int e = tid; e < H * R; e += kThreads) {
      const int r = e / H, h = e % H;
      if (r < nr) p.pool[((size_t)(k + 1) * B + i0 + r) * H + h] = NL[h * R + r];
    }
    if (p.rec_dec && tid < nr) {
      p.rec_dec[((size_t)k * B + i0 + tid) * 2] = s_r[tid];
      p.rec_dec[((size_t)k * B + i0 + tid) * 2 + 1] = s_v[tid];
      for (int a = 0; a < A; ++a) p.rec_logits[((size_t)k * B + i0 + tid) * A + a] = X1[tid * A + a];
    }
    LZM_STAMP(8);
    // ---- expand + backup (cbatch_backpropagate, cnode.cpp:480-500)
    if (tid < nr) {
      const int li = tid;
      const TreeView &tv = t;
      const int ti = tix(li);
      const int len = s_len[li];
      // best_action along the final path (cnode.cpp:806)
      for (int l = 0; l < len; ++l) tv.meta[nidx(tv, tv.path[l * R + li], ti)].best = tv.path_act[l * R + li];
      const int leaf = tv.path[len * R + li];
      int vtp = s_vtp[li];
      if (players > 1)
        for (int l = 0; l < len; ++l) vtp = (vtp == 1) ? 2 : 1;
      expand_leaf(tv, ti, leaf, vtp, k + 1, s_r[li], X1 + li * A, 0, false);
      backup_slice<false>(tv, ti, li, R, &s_mm[li], vtp, s_v[li], p.disc);
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
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)G - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace lzm
