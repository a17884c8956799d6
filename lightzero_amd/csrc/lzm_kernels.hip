// lzm_kernels.hip — MI355X (gfx950) batched MuZero / EfficientZero search tree.
//
// Replaces LightZero's ctree (lzero/mcts/ctree/ctree_{muzero,efficientzero}) and the per-
// simulation glue of lzero/mcts/tree_search/mcts_ctree.py with device kernels over a
// structure-of-arrays tree held in HBM. C ABI: include/lzmcts.h.
//
// Layout (per handle, B roots, A actions, node capacity C = 1 + A*(S_cap+1)):
//   stat[node][root]  16 B {visit, value_sum, prior, reward|value_prefix}
//   meta[node][root]  16 B {latent index (-1 = not expanded), to_play, best_action, is_reset}
// node-major with the root index fastest, so lanes of a wave that sit on the same node id
// (the root, its children) read one contiguous 1 KiB line per wave instruction. The node
// expanded with latent index L (root 0, simulation k's leaf k+1) owns children
// [1 + A*L, 1 + A*L + A) — the reference's std::map<int,CNode> children (cnode.h:26)
// without allocation. Search paths of the last traverse: path[level][root].
//
// Arithmetic follows the reference expression by expression in fp32 (compiled with
// -ffp-contract=off, IEEE division/sqrt), expf is the glibc port of lzm_numerics.h, and
// log((N+base+1)/base)+init and sqrt(N) over the integer parent count N come from a host
// table built with the host's libm (the very functions the reference calls).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <random>
#include <vector>

#include "../../include/lzmcts.h"
#include "lzm_numerics.h"
#include "lzm_collect.h"
#include "lzm_atari.h"
#include "lzm_traj.h"
#include "lzm_az.h"
#include "lzm_az_fused.h"
#include "lzm_tree.h"
#include "lzm_search_mlp.h"
#include "lzm_search_res.h"
#include "lzm_conv.h"
#include "lzm_repr.h"
#include "lzm_heads.h"
#include "lzm_lstm.h"
#include "lzm_initial.h"

namespace lzm {

struct TraverseArgs {
  TreeView t;
  const float4 *minmax;
  const uint32_t *seed;
  const int32_t *vtp_in;
  int32_t *out_x, *out_y, *out_a, *out_vtp, *out_len;
  long long *out_a64;
  uint32_t *stream;  // raw glibc stream values (before >> 1)
  int stream_cap;
  const uint32_t *jfirst;  // [kMaxWG][31]
  const uint32_t *jnext;   // [kMaxWG][31]
  int32_t *off;            // [B]
  int32_t *diag;           // [0] fixed-point passes of the last call ([1] unused: failures go to err)
  int32_t *err;            // sticky error counters (lzm_check_errors): [2] fixed point not reached
  int32_t *hint;           // [0] stream length used by the previous call
  float disc;
};

__device__ inline int block_players(const int32_t *vtp, int B) {
  // players = (max(virtual_to_play) == -1) ? 1 : 2  (cnode.cpp:776-781)
  __shared__ int s_max;
  if (threadIdx.x == 0) s_max = INT_MIN;
  __syncthreads();
  int m = INT_MIN;
  for (int i = threadIdx.x; i < B; i += blockDim.x) m = max(m, vtp[i]);
  atomicMax(&s_max, m);
  __syncthreads();
  int p = (s_max == -1) ? 1 : 2;
  __syncthreads();
  return p;
}

// Block-wide exclusive scan (blockDim multiple of 64, <= 1024).
__device__ inline int block_excl_scan(int v, int *s_w, int &total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  if (wid == 0) {
    int w = lane < nw ? s_w[lane] : 0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      int y = __shfl_up(w, d, 64);
      if (lane >= d) w += y;
    }
    if (lane < nw) s_w[lane] = w;
  }
  __syncthreads();
  const int pre = wid > 0 ? s_w[wid - 1] : 0;
  total = s_w[nw - 1];
  __syncthreads();
  return pre + x - v;
}

// Parity-mode traverse: ONE workgroup walks every root, because the reference consumes one
// process-wide rand() stream in root order (root i's draws start at sum_{j<i} depth_j).
// The walk is speculative: descend every root with assumed offsets, scan the depths, and
// repeat until the offsets reproduce themselves (the unique fixed point = the serial
// order). A tie among unexpanded children never changes a depth, so two passes is typical.
// The glibc stream is produced 1 block-width at a time by a jump matrix over Z/2^32:
// z[n+m] = sum_j J[m][j] * z[n-31+j] (random_r is linear in its 31-word state).
template <bool EZ>
__global__ __launch_bounds__(1024) void traverse_glibc_kernel(TraverseArgs p) {
  const TreeView &t = p.t;
  const int W = blockDim.x, tid = threadIdx.x, B = t.B;
  __shared__ uint32_t s_win[31];
  __shared__ uint32_t s_z0[31];
  __shared__ uint32_t s_tail[31];
  __shared__ int s_w[16];
  __shared__ int s_flag;
  const int players = block_players(p.vtp_in, B);
  if (tid == 0) glibc_seed_state(*p.seed, s_z0);
  uint32_t jn[31];
#pragma unroll
  for (int j = 0; j < 31; ++j) jn[j] = p.jnext[tid * 31 + j];
  __syncthreads();
  int generated = 0;
  auto gen_chunk = [&]() {
    uint32_t v = 0;
    if (generated == 0) {
#pragma unroll
      for (int j = 0; j < 31; ++j) v += p.jfirst[tid * 31 + j] * s_z0[j];
    } else {
#pragma unroll
      for (int j = 0; j < 31; ++j) v += jn[j] * s_win[j];
    }
    if (generated + tid < p.stream_cap) p.stream[generated + tid] = v;
    if (tid >= W - 31) s_tail[tid - (W - 31)] = v;
    __syncthreads();
    if (tid < 31) s_win[tid] = s_tail[tid];
    generated += W;
    __syncthreads();
  };
  // first chunk(s): enough for the previous call's total
  int want = *p.hint + W;
  if (want > p.stream_cap) want = p.stream_cap;
  do {
    gen_chunk();
  } while (generated < want);

  const int rounds = (B + W - 1) / W;
  for (int r = 0; r < rounds; ++r) {
    int i = r * W + tid;
    if (i < B) p.off[i] = 0;
  }
  __syncthreads();
  int passes = 0;
  for (;;) {
    ++passes;
    if (tid == 0) s_flag = 0;
    __syncthreads();
    int carry = 0, overflow = 0, changed = 0;
    for (int r = 0; r < rounds; ++r) {
      const int i = r * W + tid;
      int depth = 0;
      if (i < B) {
        const int off = p.off[i];
        const int gen = generated;
        const uint32_t *st = p.stream;
        auto draw = [&](int level) -> uint32_t {
          const int pos = off + level;
          if (pos < gen) return st[pos] >> 1;
          overflow = 1;
          return 0u;
        };
        Descent d = descend<EZ>(t, i, p.minmax[i], players, p.vtp_in[i], p.disc, draw);
        depth = d.len;
        p.out_x[i] = d.x;
        p.out_y[i] = i;
        p.out_a[i] = d.action;
        if (p.out_a64) p.out_a64[i] = d.action;
        p.out_vtp[i] = d.vtp;
        p.out_len[i] = d.len;
        t.pathlen[i] = d.len;
      }
      int total;
      const int ex = block_excl_scan(depth, s_w, total);
      if (i < B) {
        const int noff = carry + ex;
        if (noff != p.off[i]) changed = 1;
        p.off[i] = noff;
      }
      carry += total;
    }
    if (changed || overflow) s_flag = 1;  // benign race: every writer stores 1
    __syncthreads();
    const int again = s_flag;
    __syncthreads();
    if (carry > generated && generated < p.stream_cap) {
      while (generated < carry && generated < p.stream_cap) gen_chunk();
    }
    if (!again) {
      if (tid == 0) *p.hint = carry;
      break;
    }
    if (passes > B + 2) {  // cannot happen: the fixed point is reached in <= B+1 passes
      if (tid == 0) atomicAdd(p.err + 2, 1);
      break;
    }
  }
  // commit best_action along the final paths (cnode.cpp:806)
  for (int r = 0; r < rounds; ++r) {
    const int i = r * W + tid;
    if (i >= B) continue;
    const int len = t.pathlen[i];
    for (int l = 0; l < len; ++l) {
      const int node = t.path[(size_t)l * B + i];
      t.meta[nidx(t, node, i)].best = t.path_act[(size_t)l * B + i];
    }
  }
  if (tid == 0) p.diag[0] = passes;
}

// Fast-mode traverse: roots are independent (Philox4x32-10 draw per (seed, root, level)), so
// one lane per root over as many workgroups as needed.
template <bool EZ>
__global__ __launch_bounds__(256) void traverse_fast_kernel(TraverseArgs p) {
  const TreeView &t = p.t;
  const int players = block_players(p.vtp_in, t.B);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.B) return;
  const uint32_t seed = *p.seed;
  auto draw = [&](int level) -> uint32_t {
    uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)i, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
    return o.x >> 1;
  };
  Descent d = descend<EZ>(t, i, p.minmax[i], players, p.vtp_in[i], p.disc, draw);
  p.out_x[i] = d.x;
  p.out_y[i] = i;
  p.out_a[i] = d.action;
  if (p.out_a64) p.out_a64[i] = d.action;
  p.out_vtp[i] = d.vtp;
  p.out_len[i] = d.len;
  t.pathlen[i] = d.len;
  for (int l = 0; l < d.len; ++l) {
    const int node = t.path[(size_t)l * t.B + i];
    t.meta[nidx(t, node, i)].best = t.path_act[(size_t)l * t.B + i];
  }
}



struct BackpropArgs {
  TreeView t;
  float4 *minmax;
  const float *rewards, *values, *logits;
  const int32_t *to_play, *is_reset;
  int cur;
  float disc;
  const int32_t *reuse_action;  // optional: search-with-reuse, see reuse_leaf
  const float *reuse_value;
};

// cbatch_backpropagate_with_reuse (ctree_muzero/lib/cnode.cpp:502-546; EfficientZero
// ctree_efficientzero/lib/cnode.cpp:603-641, there with is_reset set on every leaf) for root i whose walk ended
// at `leaf` after `len` levels: no inference when the walk stopped on an expanded node (the root
// child of the true action: no expand, back up the reuse value); a walk that stopped at the
// unexpanded true-action child expands it but backs up the reuse value too.
__device__ inline void reuse_leaf(const TreeView &t, int i, int leaf, int len, const int32_t *ra, const float *rv,
                                  bool *no_inference, float *value) {
  *no_inference = false;
  if (!ra) return;
  const bool expanded = t.meta[nidx(t, leaf, i)].latent >= 0;
  const bool reuse = !expanded && len == 1 && t.path_act[i] == ra[i];
  if (expanded || reuse) *value = rv[i];
  *no_inference = expanded;
}

template <bool EZ>
__global__ __launch_bounds__(256) void backprop_kernel(BackpropArgs p) {
  const TreeView &t = p.t;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.B) return;
  const int len = t.pathlen[i];
  const int leaf = t.path[(size_t)len * t.B + i];
  const int tp = p.to_play[i];
  float v = p.values[i];
  bool no_inf;
  reuse_leaf(t, i, leaf, len, p.reuse_action, p.reuse_value, &no_inf, &v);
  if (!no_inf)
    expand_leaf(t, i, leaf, tp, p.cur, p.rewards[i], p.logits + (size_t)i * t.A, p.is_reset ? p.is_reset[i] : 0, EZ);
  else if (EZ)  // the reference sets every leaf's is_reset, expanded or not (ctree_efficientzero cnode.cpp:638)
    t.meta[nidx(t, leaf, i)].is_reset = p.is_reset ? p.is_reset[i] : 0;
  backup<EZ>(t, i, p.minmax + i, tp, v, p.disc);
}

// InverseScalarTransform (scaling_transform.py:118-128) of one row by one wave:
// softmax (unless `raw`), expectation over support [-(V-1)/2 .. (V-1)/2], then h^-1.
// Register form for V <= 64 * NPL: the row is loaded once, every load in flight together (the loop
// form re-reads it in three passes with one memory latency per iteration). Same per-lane order and
// the same reductions, so the same bits.
template <int NPL>
__device__ inline float wave_support_expectation_reg(const float *row, int V, bool softmax) {
  const int lane = threadIdx.x & 63;
  const float half = (float)((V - 1) / 2);
  float x[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int j = lane + 64 * q;
    x[q] = j < V ? row[j] : 0.0f;
  }
  if (!softmax) {
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < NPL; ++q)
      if (lane + 64 * q < V) acc += x[q] * ((float)(lane + 64 * q) - half);
    acc = xor_sum(acc);
    return acc;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < V) mx = fmaxf(mx, x[q]);
  mx = xor_max(mx);
  float sum = 0.0f;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < V) sum += expf(x[q] - mx);
  sum = xor_sum(sum);
  float acc = 0.0f;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < V) acc += (expf(x[q] - mx) / sum) * ((float)(lane + 64 * q) - half);
  acc = xor_sum(acc);
  return acc;
}

__device__ inline float wave_support_expectation_loop(const float *row, int V, bool softmax);

__device__ inline float wave_support_expectation(const float *row, int V, bool softmax) {
  if (V <= 64 * 2) return wave_support_expectation_reg<2>(row, V, softmax);
  if (V <= 64 * 10) return wave_support_expectation_reg<10>(row, V, softmax);
  if (V <= 64 * 16) return wave_support_expectation_reg<16>(row, V, softmax);
  return wave_support_expectation_loop(row, V, softmax);
}

__device__ inline float wave_support_expectation_loop(const float *row, int V, bool softmax) {
  const int lane = threadIdx.x & 63;
  const float half = (float)((V - 1) / 2);
  if (!softmax) {
    float acc = 0.0f;
    for (int j = lane; j < V; j += 64) acc += row[j] * ((float)j - half);
    acc = xor_sum(acc);
    return acc;
  }
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


__device__ inline float wave_row_sum(const float *row, int V) {
  const int lane = threadIdx.x & 63;
  float s = 0.0f;
  if (V <= 64 * 10) {
    // every load in flight together; same per-lane order as the loop
    float x[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) x[q] = lane + 64 * q < V ? row[lane + 64 * q] : 0.0f;
#pragma unroll
    for (int q = 0; q < 10; ++q)
      if (lane + 64 * q < V) s += x[q];
    s = xor_sum(s);
    return s;
  }
  for (int j = lane; j < V; j += 64) s += row[j];
  s = xor_sum(s);
  return s;
}

struct DecodeArgs {
  TreeView t;
  float4 *minmax;
  const float *reward_logits, *value_logits, *policy_logits;
  const int32_t *to_play;
  int32_t *out_is_reset;
  const float *next_latent;
  float *pool_slot;
  long long row_elems;
  int V, categorical, cur, horizon;
  float disc;
  float *out_decoded;  // [B][2] {reward, value} after h^-1, optional
  const int32_t *reuse_action;  // optional: search-with-reuse, see reuse_leaf
  const float *reuse_value;
};

// ensure_softmax (scaling_transform.py:36-62): softmax is skipped only when EVERY row of the
// batch already sums to 1 within allclose(atol=1e-5, rtol=1e-5) — judged per tensor (the
// reference calls the transform once per head: a = reward rows, b = value rows). Each workgroup
// (4 rows) overwrites its own verdict words part[2 * block + head] (1: no row of that head in the
// block fails), so nothing has to be cleared between calls; consumers AND the words (norm_ok).
__global__ __launch_bounds__(256) void normalized_check_kernel(const float *a, const float *b, int rows, int V,
                                                               int32_t *part) {
  __shared__ int s_ok[2];
  if (threadIdx.x == 0) s_ok[0] = s_ok[1] = 1;
  __syncthreads();
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (w < 2 * rows) {
    const float *row = (w < rows) ? a + (size_t)w * V : b + (size_t)(w - rows) * V;
    const float s = wave_row_sum(row, V);
    if ((threadIdx.x & 63) == 0 && !(fabsf(s - 1.0f) <= 1e-5f + 1e-5f)) atomicAnd(&s_ok[w < rows ? 0 : 1], 0);
  }
  __syncthreads();
  if (threadIdx.x < 2) part[2 * blockIdx.x + threadIdx.x] = s_ok[threadIdx.x];
}
__host__ __device__ inline int norm_parts(int rows) { return (2 * rows * 64 + 255) / 256; }
// head's verdict over every block's word (wave-uniform result)
__device__ inline bool norm_ok(const int32_t *part, int nparts, int head) {
  int bad = 0;
  for (int q = (threadIdx.x & 63); q < nparts; q += 64) bad |= part[2 * q + head] == 0;
  return __ballot(bad) == 0ull;
}

// decode + expand + backup of root i by one wave (all 64 lanes call it)
template <bool EZ>
__device__ inline void decode_root(const DecodeArgs &p, const int32_t *norm_part, int i) {
  const TreeView &t = p.t;
  const int lane = threadIdx.x & 63;
  // new latent row into the pool slot (mcts_ctree.py:305)
  if (p.next_latent && p.pool_slot) {
    const float *src = p.next_latent + (size_t)i * p.row_elems;
    float *dst = p.pool_slot + (size_t)i * p.row_elems;
    for (long long e = lane; e < p.row_elems; e += 64) dst[e] = src[e];
  }
  float r, v;
  if (p.categorical) {
    const int np = norm_parts(t.B);
    r = wave_support_expectation(p.reward_logits + (size_t)i * p.V, p.V, !norm_ok(norm_part, np, 0));
    v = wave_support_expectation(p.value_logits + (size_t)i * p.V, p.V, !norm_ok(norm_part, np, 1));
  } else {
    r = p.reward_logits[(size_t)i * p.V];
    v = p.value_logits[(size_t)i * p.V];
  }
  r = h_inverse(r);
  v = h_inverse(v);
  if (p.out_decoded && lane == 0) {
    p.out_decoded[2 * i] = r;
    p.out_decoded[2 * i + 1] = v;
  }
  if (t.A <= 64) {
    // one lane per child / path level, bit-identical to the serial form below (lzm_tree.h)
    const int len = t.pathlen[i];
    const int leaf = t.path[(size_t)len * t.B + i];
    const int tp = p.to_play[i];
    const int is_reset = (EZ && p.horizon > 0 && len % p.horizon == 0) ? 1 : 0;
    if (p.out_is_reset && lane == 0) p.out_is_reset[i] = is_reset;
    bool no_inf;
    reuse_leaf(t, i, leaf, len, p.reuse_action, p.reuse_value, &no_inf, &v);
    if (!no_inf) expand_wave(t, i, leaf, tp, p.cur, r, p.policy_logits + (size_t)i * t.A, EZ ? is_reset : -1);
    else if (EZ && lane == 0) t.meta[nidx(t, leaf, i)].is_reset = is_reset;  // (cnode.cpp:638, every leaf)
    if (EZ)
      backup_wave_ez(t, i, i, t.B, p.minmax + i, tp, v, p.disc);
    else
      backup_wave(t, i, i, t.B, p.minmax + i, tp, v, p.disc);
    return;
  }
  if (lane != 0) return;
  const int len = t.pathlen[i];
  const int leaf = t.path[(size_t)len * t.B + i];
  int is_reset = 0;
  if (EZ && p.horizon > 0) is_reset = (len % p.horizon == 0) ? 1 : 0;
  if (p.out_is_reset) p.out_is_reset[i] = is_reset;
  const int tp = p.to_play[i];
  bool no_inf;
  reuse_leaf(t, i, leaf, len, p.reuse_action, p.reuse_value, &no_inf, &v);
  if (!no_inf) expand_leaf(t, i, leaf, tp, p.cur, r, p.policy_logits + (size_t)i * t.A, is_reset, EZ);
  else if (EZ) t.meta[nidx(t, leaf, i)].is_reset = is_reset;
  backup<EZ>(t, i, p.minmax + i, tp, v, p.disc);
}

template <bool EZ>
__global__ __launch_bounds__(256) void decode_backprop_kernel(DecodeArgs p, const int32_t *norm_part) {
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // one wave per root
  if (i < p.t.B) decode_root<EZ>(p, norm_part, i);
}

__global__ __launch_bounds__(256) void inverse_transform_kernel(const float *logits, int rows, int V, int categorical,
                                                                const int32_t *norm_part, float *out) {
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (i >= rows) return;
  float v;
  if (categorical) {
    v = wave_support_expectation(logits + (size_t)i * V, V, !norm_ok(norm_part, norm_parts(rows), 0));
  } else {
    v = logits[(size_t)i * V];
  }
  if ((threadIdx.x & 63) == 0) out[i] = h_inverse(v);
}


__global__ __launch_bounds__(256) void prepare_kernel(PrepareArgs p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < p.B) prepare_root(p, i);
}

__global__ void minmax_init_kernel(float4 *mm, int n, float delta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mm[i] = make_float4(kFloatMin, kFloatMax, delta, 0.0f);
}

// collect-step mode on the weight-streaming path (the network-resident kernel does both in-kernel):
// seeds of this step (seed_sequence_kernel's rule) and, optionally, fresh min-max bounds ...
__global__ void step_prologue_kernel(const int64_t *count, long long base, int S, int32_t *seeds, float4 *mm, int n,
                                     int fresh, float delta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (count && i < S) seeds[i] = (int32_t)((base + *count * (long long)S + i) % 1000000ll);
  if (fresh && i < n) mm[i] = make_float4(kFloatMin, kFloatMax, delta, 0.0f);
}

__global__ void gather_kernel(const float *pool, long long row, int B, const int32_t *x, float *out) {
  const long long total = (long long)B * row;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e / row);
    const long long c = e - (long long)i * row;
    const int xi = max(x[i], 0);
    out[e] = pool[((long long)xi * B + i) * row + c];
  }
}

__global__ void gather_kernel_v4(const float4 *pool, long long row4, int B, const int32_t *x, float4 *out) {
  const long long total = (long long)B * row4;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e / row4);
    const long long c = e - (long long)i * row4;
    const int xi = max(x[i], 0);  // an unexpanded root reports -1 (reference: UB); never read before the pool
    out[e] = pool[((long long)xi * B + i) * row4 + c];
  }
}

__global__ void distributions_kernel(TreeView t, int32_t *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.B) return;
  const NodeMeta rm = t.meta[i];
  for (int j = 0; j < t.A; ++j) {
    int v = -1;
    if (rm.latent >= 0 && j < t.nlegal[i]) v = t.stat[nidx(t, 1 + t.A * rm.latent + t.legal[(size_t)i * t.A + j], i)].visit;
    out[(size_t)i * t.A + j] = v;
  }
}

// get_distributions and get_values in one pass (the collect step reads both every env step)
__global__ void root_outputs_kernel(TreeView t, int32_t *dist, float *values) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.B) return;
  const NodeStat rs = t.stat[i];
  const NodeMeta rm = t.meta[i];
  for (int j = 0; j < t.A; ++j) {
    int v = -1;
    if (rm.latent >= 0 && j < t.nlegal[i]) v = t.stat[nidx(t, 1 + t.A * rm.latent + t.legal[(size_t)i * t.A + j], i)].visit;
    dist[(size_t)i * t.A + j] = v;
  }
  values[i] = node_value(rs);
}

// ... and after the search: the root outputs (root_outputs_kernel) and the step counter
__global__ void step_epilogue_kernel(TreeView t, int32_t *dist, float *values, int64_t *count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (dist && i < t.B) {
    const NodeMeta rm = t.meta[i];
    for (int j = 0; j < t.A; ++j) {
      int v = -1;
      if (rm.latent >= 0 && j < t.nlegal[i]) v = t.stat[nidx(t, 1 + t.A * rm.latent + t.legal[(size_t)i * t.A + j], i)].visit;
      dist[(size_t)i * t.A + j] = v;
    }
  }
  if (values && i < t.B) values[i] = node_value(t.stat[i]);
  if (count && i == 0) *count += 1;
}

__global__ void values_kernel(TreeView t, float *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < t.B) out[i] = node_value(t.stat[i]);
}

__global__ void trajectories_kernel(TreeView t, int32_t *out, int tmax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.B) return;
  int node = 0, n = 0;
  NodeMeta m = t.meta[nidx(t, 0, i)];
  while (m.best >= 0 && n < tmax && m.latent >= 0) {
    out[(size_t)i * tmax + n++] = m.best;
    node = 1 + t.A * m.latent + m.best;
    m = t.meta[nidx(t, node, i)];
  }
  for (; n < tmax; ++n) out[(size_t)i * tmax + n] = -1;
}

__global__ void debug_expf_kernel(const float *x, float *out, long long n) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    out[e] = glibc_expf(x[e]);
}

// lzm_debug_xor: the DPP / permlane butterfly helpers (lzm_tree.h xor_partner / xor_sum / xor_max) beside
// the ds_bpermute __shfl_xor they replace, one 64-lane wave; rows of out [16][64]:
//   0-5 xor_partner<1..32>, 6-11 __shfl_xor(v, 1..32), 12 xor_sum, 13 the __shfl_xor butterfly sum,
//   14 xor_max, 15 the __shfl_xor butterfly max
__global__ void __launch_bounds__(64) debug_xor_kernel(const float *in, float *out) {
  const int l = threadIdx.x;
  const float v = in[l];
  out[0 * 64 + l] = xor_partner<1>(v);
  out[1 * 64 + l] = xor_partner<2>(v);
  out[2 * 64 + l] = xor_partner<4>(v);
  out[3 * 64 + l] = xor_partner<8>(v);
  out[4 * 64 + l] = xor_partner<16>(v);
  out[5 * 64 + l] = xor_partner<32>(v);
  for (int k = 0; k < 6; ++k) out[(6 + k) * 64 + l] = __shfl_xor(v, 1 << k, 64);
  out[12 * 64 + l] = xor_sum(v);
  float s = v, m = v;
  for (int d = 32; d >= 1; d >>= 1) {
    s += __shfl_xor(s, d, 64);
    m = fmaxf(m, __shfl_xor(m, d, 64));
  }
  out[13 * 64 + l] = s;
  out[14 * 64 + l] = xor_max(v);
  out[15 * 64 + l] = m;
}

// lzm_debug_az_rules: the fused AlphaZero search's mask / DPP forms beside the scans they replace, one board per
// 16-lane group: out[b][6] = {done, winner by az_done_winner (the reference's cell scan), done, winner by
// az_done_winner_mask, the lane az_group_argmax picks from scores[b][16], the first strict maximum of a scan}
__global__ void __launch_bounds__(64) debug_az_rules_kernel(int n, const int32_t *boards, const double *scores,
                                                            int32_t *out) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 4), l = threadIdx.x & 15, gbase = (threadIdx.x & 63) & ~15;
  const bool on = b < n;  // group-uniform
  const int cell = on && l < 9 ? boards[(size_t)b * 9 + l] : 0;
  const double sc = on ? scores[(size_t)b * 16 + l] : 0.0;
  const int bi = az_group_argmax(sc, gbase);  // (every lane of the wave takes part)
  int done_m, win_m;
  az_done_winner_mask(az_group_mask(l < 9 && cell == 1, gbase), az_group_mask(l < 9 && cell == 2, gbase), done_m, win_m);
  if (!on || l != 0) return;
  int bd[9];
  for (int k = 0; k < 9; ++k) bd[k] = boards[(size_t)b * 9 + k];
  int done_s, win_s;
  az_done_winner(bd, done_s, win_s);
  int best = 0;
  for (int k = 1; k < 16; ++k)
    if (scores[(size_t)b * 16 + k] > scores[(size_t)b * 16 + best]) best = k;
  int32_t *o = out + (size_t)b * 6;
  o[0] = done_s; o[1] = win_s; o[2] = done_m; o[3] = win_m; o[4] = bi; o[5] = best;
}

__global__ void debug_philox_kernel(const uint32_t *ck, uint32_t *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t *c = ck + (size_t)i * 6;
  uint4 o = philox4x32_10(make_uint4(c[0], c[1], c[2], c[3]), make_uint2(c[4], c[5]));
  out[(size_t)i * 4 + 0] = o.x;
  out[(size_t)i * 4 + 1] = o.y;
  out[(size_t)i * 4 + 2] = o.z;
  out[(size_t)i * 4 + 3] = o.w;
}

__global__ void debug_glibc_kernel(uint32_t seed, int n, int32_t *out, const uint32_t *jfirst, const uint32_t *jnext) {
  // single workgroup; exercises the same jump-matrix generator as traverse_glibc_kernel
  __shared__ uint32_t s_z0[31], s_win[31], s_tail[31];
  const int W = blockDim.x, tid = threadIdx.x;
  if (tid == 0) glibc_seed_state(seed, s_z0);
  __syncthreads();
  for (int g = 0; g < n; g += W) {
    uint32_t v = 0;
    for (int j = 0; j < 31; ++j) v += (g == 0 ? jfirst[tid * 31 + j] * s_z0[j] : jnext[tid * 31 + j] * s_win[j]);
    if (g + tid < n) out[g + tid] = (int32_t)(v >> 1);
    if (tid >= W - 31) s_tail[tid - (W - 31)] = v;
    __syncthreads();
    if (tid < 31) s_win[tid] = s_tail[tid];
    __syncthreads();
  }
}

}  // namespace lzm

#include "lzm_traverse_lb.h"  // uses block_players above
#include "lzm_search_conv.h"  // uses wave_support_expectation / wave_row_sum above

namespace lzm {

// Simulation k's decode + expand + backup fused with simulation k + 1's traverse (generic search
// path, parity mode): the wave that backs up root i walks root i again at once, over the records it
// has just written (warm in this CU's caches) and without a launch of its own. The walk is the
// look-back traverse's (lzm_traverse_lb.h), so requests and draws are those of the separate launches.
template <bool EZ>
__global__ __launch_bounds__(kTlbThreads) void decode_traverse_kernel(DecodeArgs p, const int32_t *norm_part,
                                                                      TraverseLbArgs q) {
  __shared__ uint32_t s_z0[31], s_pow[31];
  __shared__ int s_epoch;
  int players;
  const unsigned long long epoch = traverse_lb_setup(q, s_z0, s_pow, &s_epoch, &players);
  const int i = blockIdx.x * (kTlbThreads / 64) + (threadIdx.x >> 6);
  if (i < p.t.B) {
    decode_root<EZ>(p, norm_part, i);
    // the backup's stores (other lanes of this wave) complete before the walk reads them; the walk
    // runs on the same CU, so workgroup scope suffices (agent scope would write back the L2)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    traverse_lb_root<EZ>(q, i, s_z0, epoch, players);
  }
  traverse_lb_finish(q, epoch);
}

}  // namespace lzm

// ============================================================================ host side
using namespace lzm;

static thread_local char g_err[512];
constexpr int kErrWords = 8;  // sticky error words per handle (lzm_check_errors)
static void set_err(const char *msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }
#define LZM_HIP(call)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      snprintf(g_err, sizeof(g_err), "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
      return LZM_ERR_HIP;                                                                          \
    }                                                                                              \
  } while (0)
#define LZM_CHECK_LAUNCH() LZM_HIP(hipGetLastError())

// Compute units of the CURRENT device, cached per device ordinal (a process may drive several GPUs,
// or switch devices between calls: a process-wide static would keep the first device's count).
static int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev >= 64) {
    int n = 0;
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  if (!cache[dev]) {
    int n = 0;
    cache[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return cache[dev];
}

struct lzm_handle {
  int B, A, flags, sims_cap, cap, depth_cap;
  NodeStat *stat = nullptr;
  NodeMeta *meta = nullptr;
  int32_t *legal = nullptr, *nlegal = nullptr, *path = nullptr, *path_act = nullptr, *pathlen = nullptr;
  int32_t *off = nullptr, *diag = nullptr, *hint = nullptr, *norm_flag = nullptr;
  int32_t *err = nullptr;  // [4] sticky error counters of the generic path (lzm_check_errors)
  uint32_t *stream = nullptr;
  int stream_cap = 0;
  float2 *lut = nullptr;
  int lut_n = 0;
  int lut_base = -1;
  float lut_init = -1.0f;
  uint32_t *jmat = nullptr;  // [2][kMaxWG][31]
  // fused whole-search state (lzm_search_mlp)
  uint32_t *coef = nullptr;  // [coef_positions][31] glibc draw coefficients
  int coef_positions = 0;
  uint32_t *pow16807 = nullptr;            // [31]
  unsigned long long *lb_flags = nullptr;  // [flag_sims][G] look-back words
  int flag_sims = 0;
  uint32_t *epoch = nullptr;               // [2] launch epoch, done counter
  int32_t *search_diag = nullptr;          // [4]
  // collect-step mode of the fused search (lzm_search_set_step)
  int64_t *step_count = nullptr;
  int step_inc = 0;
  long long step_base = 0;
  int step_fresh = 0;
  float step_delta = 0.0f;
  int32_t *step_dist = nullptr;
  float *step_vals = nullptr;
  int32_t *step_seeds = nullptr;  // [sims] the weight-streaming path's staged seeds
  int step_seeds_n = 0;
  unsigned long long *phase = nullptr;     // [64] diagnostic phase cycles (LZM_PHASE_TIMING=1)
  const int32_t *ext_norm = nullptr;       // lzm_set_norm_words: verdict words written by lzm_conv_heads
  const int32_t *reuse_action = nullptr;   // lzm_set_reuse: search-with-reuse inputs (device, [B])
  const float *reuse_value = nullptr;
  // lzm_search_conv_ez's hand-off workspace (LSTM input rows, outputs, split-K partials, flags)
  void *ez_ws = nullptr;
  size_t ez_ws_bytes = 0;
};

// Jump matrices of glibc random_r: row m of J_first expresses z[344+m] (the m-th rand()
// output before >>1) in the 31-word seeded state; row m of J_next expresses z[n+m] in the
// window z[n-31..n-1]. Coefficients over Z/2^32 (wrapping uint32 arithmetic).
static void build_jump_matrices(std::vector<uint32_t> &jf, std::vector<uint32_t> &jn) {
  const int W = kMaxWG;
  jf.assign((size_t)W * 31, 0u);
  jn.assign((size_t)W * 31, 0u);
  {
    const int N = 344 + W;
    std::vector<uint32_t> z((size_t)N * 31, 0u);
    for (int j = 0; j < 31; ++j) z[(size_t)j * 31 + j] = 1u;
    for (int j = 31; j < 34; ++j)
      for (int c = 0; c < 31; ++c) z[(size_t)j * 31 + c] = z[(size_t)(j - 31) * 31 + c];
    for (int n = 34; n < N; ++n)
      for (int c = 0; c < 31; ++c) z[(size_t)n * 31 + c] = z[(size_t)(n - 31) * 31 + c] + z[(size_t)(n - 3) * 31 + c];
    for (int m = 0; m < W; ++m)
      for (int c = 0; c < 31; ++c) jf[(size_t)m * 31 + c] = z[(size_t)(344 + m) * 31 + c];
  }
  {
    const int N = 31 + W;
    std::vector<uint32_t> z((size_t)N * 31, 0u);
    for (int j = 0; j < 31; ++j) z[(size_t)j * 31 + j] = 1u;
    for (int n = 31; n < N; ++n)
      for (int c = 0; c < 31; ++c) z[(size_t)n * 31 + c] = z[(size_t)(n - 31) * 31 + c] + z[(size_t)(n - 3) * 31 + c];
    for (int m = 0; m < W; ++m)
      for (int c = 0; c < 31; ++c) jn[(size_t)m * 31 + c] = z[(size_t)(31 + m) * 31 + c];
  }
}

static TreeView view(lzm_handle *h) {
  TreeView t;
  t.stat = h->stat;
  t.meta = h->meta;
  t.legal = h->legal;
  t.nlegal = h->nlegal;
  t.path = h->path;
  t.path_act = h->path_act;
  t.pathlen = h->pathlen;
  t.lut = h->lut;
  t.B = h->B;
  t.A = h->A;
  t.cap = h->cap;
  t.lut_n = h->lut_n;
  t.depth_cap = h->depth_cap;
  return t;
}

static void dfree(void *p) {
  if (p) (void)hipFree(p);
}

static void free_tree(lzm_handle *h) {
  dfree(h->stat); dfree(h->meta); dfree(h->path); dfree(h->path_act); dfree(h->stream); dfree(h->lut);
  dfree(h->step_seeds);
  h->stat = nullptr; h->meta = nullptr; h->path = nullptr; h->path_act = nullptr; h->stream = nullptr; h->lut = nullptr;
  h->step_seeds = nullptr;
  h->step_seeds_n = 0;
}

// pb_c table over the integer parent count N = visit-1 (cucb_score, cnode.cpp:673-674):
// {logf(((N + base) + 1) / base) + init, sqrtf(N)} with the host libm, -ffp-contract=off.
static int fill_lut(lzm_handle *h, int base, float init) {
  if (h->lut_base == base && h->lut_init == init) return LZM_OK;
  std::vector<float2> lut(h->lut_n);
  const float fb = (float)base;
  for (int n = 0; n < h->lut_n; ++n) {
    volatile float N = (float)n;
    volatile float num = N + fb;
    num = num + 1;
    volatile float q = num / fb;
    float pbc = logf(q) + init;
    lut[n] = make_float2(pbc, sqrtf(N));
  }
  LZM_HIP(hipMemcpy(h->lut, lut.data(), sizeof(float2) * h->lut_n, hipMemcpyHostToDevice));
  h->lut_base = base;
  h->lut_init = init;
  return LZM_OK;
}

namespace {
int ensure_coef(lzm_handle *h, int positions);
int ensure_flags(lzm_handle *h, int sims, int G);
}  // namespace

static int alloc_tree(lzm_handle *h, int sims) {
  h->sims_cap = sims;
  h->cap = 1 + h->A * (sims + 1);
  h->depth_cap = sims + 2;
  const size_t nodes = (size_t)h->cap * h->B;
  LZM_HIP(hipMalloc(&h->stat, nodes * sizeof(NodeStat)));
  LZM_HIP(hipMalloc(&h->meta, nodes * sizeof(NodeMeta)));
  LZM_HIP(hipMemset(h->meta, 0xff, nodes * sizeof(NodeMeta)));  // latent -1: nothing expanded
  LZM_HIP(hipMemset(h->stat, 0, nodes * sizeof(NodeStat)));
  LZM_HIP(hipMalloc(&h->path, sizeof(int32_t) * (size_t)h->depth_cap * h->B));
  LZM_HIP(hipMalloc(&h->path_act, sizeof(int32_t) * (size_t)h->depth_cap * h->B));
  h->stream_cap = h->B * (sims + 2) + 2 * kMaxWG;
  LZM_HIP(hipMalloc(&h->stream, sizeof(uint32_t) * (size_t)h->stream_cap));
  h->lut_n = sims + 8;
  LZM_HIP(hipMalloc(&h->lut, sizeof(float2) * h->lut_n));
  h->lut_base = -1;
  // the collect-step seeds of the weight-streaming search (lzm_search_set_step): sized with the
  // tree, so a captured step never allocates and a reserve (generation bump) retires graphs that
  // point at the old buffer together with the tree's
  LZM_HIP(hipMalloc(&h->step_seeds, sizeof(int32_t) * (size_t)(sims + 1)));
  h->step_seeds_n = sims + 1;
  if (!(h->flags & LZM_RNG_FAST)) {
    // parity-mode draw tables and look-back words, allocated here rather than at first use so
    // that a search captured into a HIP graph never allocates
    int rc = ensure_coef(h, h->B * h->depth_cap + 64);
    if (rc != LZM_OK) return rc;
    rc = ensure_flags(h, sims, h->B);
    if (rc != LZM_OK) return rc;
  }
  return fill_lut(h, 19652, 1.25f);
}

extern "C" {

const char *lzm_last_error(void) { return g_err; }

int lzm_create(int B, int A, int max_sims, int flags, lzm_handle **out) {
  if (!out || B <= 0 || A <= 0 || A > kMaxActions || max_sims < 0) {
    set_err("lzm_create: need num_roots > 0, 0 < action_space <= 64, max_sims >= 0");
    return LZM_ERR_ARG;
  }
  lzm_handle *h = new lzm_handle();
  h->B = B;
  h->A = A;
  h->flags = flags;
  int rc;
#define TRY(x) do { rc = (x); if (rc != LZM_OK) { lzm_destroy(h); return rc; } } while (0)
  TRY(hipMalloc(&h->legal, sizeof(int32_t) * (size_t)B * A) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->nlegal, sizeof(int32_t) * B) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->pathlen, sizeof(int32_t) * B) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->off, sizeof(int32_t) * B) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->diag, sizeof(int32_t) * 4) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->err, sizeof(int32_t) * kErrWords) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMemset(h->err, 0, sizeof(int32_t) * kErrWords) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->hint, sizeof(int32_t) * 2) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMalloc(&h->norm_flag, sizeof(int32_t) * 2 * norm_parts(B)) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMemset(h->diag, 0, sizeof(int32_t) * 4) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMemset(h->hint, 0, sizeof(int32_t) * 2) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  TRY(hipMemset(h->pathlen, 0, sizeof(int32_t) * B) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  {
    std::vector<uint32_t> jf, jn;
    build_jump_matrices(jf, jn);
    TRY(hipMalloc(&h->jmat, sizeof(uint32_t) * 2 * kMaxWG * 31) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
    TRY(hipMemcpy(h->jmat, jf.data(), sizeof(uint32_t) * kMaxWG * 31, hipMemcpyHostToDevice) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
    TRY(hipMemcpy(h->jmat + kMaxWG * 31, jn.data(), sizeof(uint32_t) * kMaxWG * 31, hipMemcpyHostToDevice) == hipSuccess ? LZM_OK : LZM_ERR_HIP);
  }
  TRY(alloc_tree(h, max_sims));
#undef TRY
  *out = h;
  return LZM_OK;
}

int lzm_destroy(lzm_handle *h) {
  if (!h) return LZM_OK;
  free_tree(h);
  dfree(h->legal); dfree(h->nlegal); dfree(h->pathlen); dfree(h->off); dfree(h->diag); dfree(h->err);
  dfree(h->hint); dfree(h->norm_flag); dfree(h->jmat);
  dfree(h->coef); dfree(h->pow16807); dfree(h->lb_flags); dfree(h->epoch); dfree(h->search_diag); dfree(h->phase);
  dfree(h->ez_ws);
  delete h;
  return LZM_OK;
}

// Grows the node pool, keeping the tree: node-major storage means the old pool is a prefix
// of the new one (same for the [level][root] path arrays). Synchronises the device.
int lzm_reserve(lzm_handle *h, int max_sims) {
  if (!h || max_sims < 0) return LZM_ERR_ARG;
  if (max_sims <= h->sims_cap) return LZM_OK;
  LZM_HIP(hipDeviceSynchronize());
  lzm_handle old = *h;
  h->stat = nullptr; h->meta = nullptr; h->path = nullptr; h->path_act = nullptr; h->stream = nullptr; h->lut = nullptr;
  int rc = alloc_tree(h, max_sims);
  if (rc == LZM_OK) {
    const size_t nodes = (size_t)old.cap * old.B;
    LZM_HIP(hipMemcpy(h->stat, old.stat, nodes * sizeof(NodeStat), hipMemcpyDeviceToDevice));
    LZM_HIP(hipMemcpy(h->meta, old.meta, nodes * sizeof(NodeMeta), hipMemcpyDeviceToDevice));
    LZM_HIP(hipMemcpy(h->path, old.path, sizeof(int32_t) * (size_t)old.depth_cap * old.B, hipMemcpyDeviceToDevice));
    LZM_HIP(hipMemcpy(h->path_act, old.path_act, sizeof(int32_t) * (size_t)old.depth_cap * old.B, hipMemcpyDeviceToDevice));
    if (old.lut_base >= 0) rc = fill_lut(h, old.lut_base, old.lut_init);
  }
  free_tree(&old);
  return rc;
}

int lzm_set_pb_c(lzm_handle *h, int pb_c_base, float pb_c_init) {
  if (!h || pb_c_base <= 0) return LZM_ERR_ARG;
  return fill_lut(h, pb_c_base, pb_c_init);
}

int lzm_copy_tree(lzm_handle *dst, const lzm_handle *src, void *stream) {
  if (!dst || !src || dst->B != src->B || dst->A != src->A || dst->sims_cap < src->sims_cap) {
    set_err("lzm_copy_tree: handles differ in shape or destination is smaller");
    return LZM_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const size_t nodes = (size_t)src->cap * src->B;
  LZM_HIP(hipMemcpyAsync(dst->stat, src->stat, nodes * sizeof(NodeStat), hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->meta, src->meta, nodes * sizeof(NodeMeta), hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->legal, src->legal, sizeof(int32_t) * (size_t)src->B * src->A, hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->nlegal, src->nlegal, sizeof(int32_t) * src->B, hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->path, src->path, sizeof(int32_t) * (size_t)src->depth_cap * src->B, hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->path_act, src->path_act, sizeof(int32_t) * (size_t)src->depth_cap * src->B, hipMemcpyDeviceToDevice, s));
  LZM_HIP(hipMemcpyAsync(dst->pathlen, src->pathlen, sizeof(int32_t) * src->B, hipMemcpyDeviceToDevice, s));
  return LZM_OK;
}

int lzm_num_roots(const lzm_handle *h) { return h ? h->B : LZM_ERR_ARG; }
int lzm_sims_capacity(const lzm_handle *h) { return h ? h->sims_cap : LZM_ERR_ARG; }
int lzm_action_space(const lzm_handle *h) { return h ? h->A : LZM_ERR_ARG; }
int lzm_flags(const lzm_handle *h) { return h ? h->flags : LZM_ERR_ARG; }

int lzm_minmax_init(float *mm, int n, float delta, void *stream) {
  if (!mm || n <= 0) return LZM_ERR_ARG;
  hipLaunchKernelGGL(minmax_init_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (float4 *)mm, n, delta);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_roots_prepare(lzm_handle *h, const int32_t *legal, const int32_t *count, const float *noises, float noise_weight,
                      const float *rewards, const float *logits, const int32_t *to_play, void *stream) {
  if (!h || !legal || !count || !rewards || !logits || !to_play) {
    set_err("lzm_roots_prepare: null argument");
    return LZM_ERR_ARG;
  }
  PrepareArgs p;
  p.stat = h->stat; p.meta = h->meta; p.legal = h->legal; p.nlegal = h->nlegal;
  p.legal_in = legal; p.count_in = count; p.to_play = to_play; p.noises = noises; p.rewards = rewards;
  p.logits = logits; p.noise_weight = noise_weight; p.B = h->B; p.A = h->A;
  hipLaunchKernelGGL(prepare_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, p);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_traverse(lzm_handle *h, int pb_c_base, float pb_c_init, float discount, float *minmax, const uint32_t *seed,
                 const int32_t *vtp_in, int32_t *out_x, int32_t *out_y, int32_t *out_a, int64_t *out_a64,
                 int32_t *out_vtp, int32_t *out_len, void *stream) {
  if (!h || !minmax || !seed || !vtp_in || !out_x || !out_y || !out_a || !out_vtp || !out_len) {
    set_err("lzm_traverse: null argument");
    return LZM_ERR_ARG;
  }
  if (pb_c_base <= 0) {
    set_err("lzm_traverse: pb_c_base must be positive");
    return LZM_ERR_ARG;
  }
  int rc = fill_lut(h, pb_c_base, pb_c_init);
  if (rc != LZM_OK) return rc;
  TraverseArgs p;
  p.t = view(h);
  p.minmax = (const float4 *)minmax;
  p.seed = seed;
  p.vtp_in = vtp_in;
  p.out_x = out_x; p.out_y = out_y; p.out_a = out_a; p.out_vtp = out_vtp; p.out_len = out_len;
  p.out_a64 = (long long *)out_a64;
  p.stream = h->stream;
  p.stream_cap = h->stream_cap;
  p.jfirst = h->jmat;
  p.jnext = h->jmat + kMaxWG * 31;
  p.off = h->off;
  p.diag = h->diag;
  p.err = h->err;
  p.hint = h->hint;
  p.disc = discount;
  const bool ez = h->flags & LZM_TREE_EZ;
  hipStream_t s = (hipStream_t)stream;
  const bool serial = getenv("LZM_TRAVERSE") && strcmp(getenv("LZM_TRAVERSE"), "serial") == 0;
  if (h->reuse_action && ((h->flags & LZM_RNG_FAST) || serial)) {
    set_err("lzm_traverse: search-with-reuse needs parity mode with the look-back traverse");
    return LZM_ERR_ARG;
  }
  if (h->flags & LZM_RNG_FAST) {
    dim3 g((h->B + 255) / 256), b(256);
    if (ez) hipLaunchKernelGGL(traverse_fast_kernel<true>, g, b, 0, s, p);
    else hipLaunchKernelGGL(traverse_fast_kernel<false>, g, b, 0, s, p);
  } else if (!serial) {
    // one wave per root, decoupled look-back of the draw offsets (lzm_traverse_lb.h)
    rc = ensure_coef(h, h->B * h->depth_cap + 64);
    if (rc != LZM_OK) return rc;
    rc = ensure_flags(h, 1, 1);
    if (rc != LZM_OK) return rc;
    TraverseLbArgs q;
    q.t = p.t; q.minmax = p.minmax; q.seed = seed; q.vtp_in = vtp_in;
    q.out_x = out_x; q.out_y = out_y; q.out_a = out_a; q.out_vtp = out_vtp; q.out_len = out_len;
    q.out_a64 = p.out_a64; q.disc = discount;
    q.coef = h->coef; q.coef_positions = h->coef_positions; q.pow16807 = h->pow16807;
    q.flags = h->lb_flags; q.epoch = h->epoch; q.diag = h->diag; q.err = h->err;
    q.reuse_action = h->reuse_action; q.reuse_value = h->reuse_value;
    q.stamps = nullptr;
    // LZM_TLB_WAVES (experiments): roots (waves) per workgroup, 1 (default), 2 or 4
    static const int waves = getenv("LZM_TLB_WAVES") ? atoi(getenv("LZM_TLB_WAVES")) : 1;
    const int per = (waves == 2 || waves == 4) ? waves : 1;
    dim3 g((h->B + per - 1) / per), b(64 * per);
    static const bool stamps = getenv("LZM_PHASE_TIMING") && atoi(getenv("LZM_PHASE_TIMING")) > 0;
    if (stamps) {  // diagnostic instantiation: per-phase cycles into phase[32..38] (lzm_debug_phase_cycles)
      if (!h->phase) {
        LZM_HIP(hipMalloc(&h->phase, (64 + 1024) * sizeof(unsigned long long)));
        LZM_HIP(hipMemset(h->phase, 0, (64 + 1024) * sizeof(unsigned long long)));
      }
      q.stamps = h->phase;
      dim3 g1(h->B), b1(64);
      if (ez) hipLaunchKernelGGL((traverse_lookback_kernel<true, 1, true>), g1, b1, 0, s, q);
      else hipLaunchKernelGGL((traverse_lookback_kernel<false, 1, true>), g1, b1, 0, s, q);
    } else if (per == 1) {
      if (ez) hipLaunchKernelGGL((traverse_lookback_kernel<true, 1>), g, b, 0, s, q);
      else hipLaunchKernelGGL((traverse_lookback_kernel<false, 1>), g, b, 0, s, q);
    } else if (per == 2) {
      if (ez) hipLaunchKernelGGL((traverse_lookback_kernel<true, 2>), g, b, 0, s, q);
      else hipLaunchKernelGGL((traverse_lookback_kernel<false, 2>), g, b, 0, s, q);
    } else {
      if (ez) hipLaunchKernelGGL(traverse_lookback_kernel<true>, g, b, 0, s, q);
      else hipLaunchKernelGGL(traverse_lookback_kernel<false>, g, b, 0, s, q);
    }
  } else {
    // LZM_TRAVERSE=serial: one workgroup, speculative fixed-point passes over the stream
    int W = ((h->B + 63) / 64) * 64;
    if (W > kMaxWG) W = kMaxWG;
    if (W < 64) W = 64;
    if (ez) hipLaunchKernelGGL(traverse_glibc_kernel<true>, dim3(1), dim3(W), 0, s, p);
    else hipLaunchKernelGGL(traverse_glibc_kernel<false>, dim3(1), dim3(W), 0, s, p);
  }
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_gather_latent(lzm_handle *h, const float *pool, int64_t row, const int32_t *x, float *out, void *stream) {
  if (!h || !pool || !x || !out || row <= 0) return LZM_ERR_ARG;
  const long long total = (long long)h->B * row;
  hipStream_t s = (hipStream_t)stream;
  if (row % 4 == 0 && ((uintptr_t)pool % 16 == 0) && ((uintptr_t)out % 16 == 0)) {
    const long long t4 = total / 4;
    int grid = (int)((t4 + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(gather_kernel_v4, dim3(grid), dim3(256), 0, s, (const float4 *)pool, (long long)(row / 4), h->B, x,
                       (float4 *)out);
  } else {
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, s, pool, (long long)row, h->B, x, out);
  }
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static int check_cur(lzm_handle *h, int cur) {
  if (cur < 1 || 1 + h->A * (cur + 1) > h->cap) {
    snprintf(g_err, sizeof(g_err), "latent index %d outside reserved capacity (%d simulations)", cur, h->sims_cap);
    return LZM_ERR_CAPACITY;
  }
  return LZM_OK;
}

int lzm_backprop(lzm_handle *h, int cur, float discount, float *minmax, const float *rewards, const float *values,
                 const float *logits, const int32_t *to_play, const int32_t *is_reset, void *stream) {
  if (!h || !minmax || !rewards || !values || !logits || !to_play) {
    set_err("lzm_backprop: null argument");
    return LZM_ERR_ARG;
  }
  int rc = check_cur(h, cur);
  if (rc != LZM_OK) return rc;
  BackpropArgs p;
  p.t = view(h);
  p.minmax = (float4 *)minmax;
  p.rewards = rewards; p.values = values; p.logits = logits; p.to_play = to_play; p.is_reset = is_reset;
  p.cur = cur;
  p.disc = discount;
  p.reuse_action = h->reuse_action; p.reuse_value = h->reuse_value;
  dim3 g((h->B + 255) / 256), b(256);
  if (h->flags & LZM_TREE_EZ) hipLaunchKernelGGL(backprop_kernel<true>, g, b, 0, (hipStream_t)stream, p);
  else hipLaunchKernelGGL(backprop_kernel<false>, g, b, 0, (hipStream_t)stream, p);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static int launch_norm_check(lzm_handle *hflag_owner, int32_t *flag, const float *a, const float *b, int rows, int V,
                             hipStream_t s) {
  (void)hflag_owner;
  hipLaunchKernelGGL(normalized_check_kernel, dim3(norm_parts(rows)), dim3(256), 0, s, a, b, rows, V, flag);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_decode_backprop(lzm_handle *h, int cur, float discount, float *minmax, const float *reward_logits,
                        const float *value_logits, int support_len, int categorical, const float *policy_logits,
                        const int32_t *to_play, int lstm_horizon, int32_t *out_is_reset, const float *next_latent,
                        float *pool_slot, int64_t row_elems, float *out_decoded, void *stream) {
  if (!h || !minmax || !reward_logits || !value_logits || !policy_logits || !to_play || support_len <= 0) {
    set_err("lzm_decode_backprop: null argument");
    return LZM_ERR_ARG;
  }
  if (categorical && support_len % 2 == 0) {
    set_err("lzm_decode_backprop: categorical support length must be odd (2*support_scale+1)");
    return LZM_ERR_ARG;
  }
  int rc = check_cur(h, cur);
  if (rc != LZM_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (categorical && !h->ext_norm) {
    rc = launch_norm_check(h, h->norm_flag, reward_logits, value_logits, h->B, support_len, s);
    if (rc != LZM_OK) return rc;
  }
  DecodeArgs p;
  p.t = view(h);
  p.minmax = (float4 *)minmax;
  p.reward_logits = reward_logits; p.value_logits = value_logits; p.policy_logits = policy_logits;
  p.to_play = to_play; p.out_is_reset = out_is_reset; p.next_latent = next_latent; p.pool_slot = pool_slot;
  p.row_elems = row_elems; p.V = support_len; p.categorical = categorical; p.cur = cur; p.horizon = lstm_horizon;
  p.disc = discount; p.out_decoded = out_decoded;
  p.reuse_action = h->reuse_action; p.reuse_value = h->reuse_value;
  dim3 g((h->B * 64 + 255) / 256), b(256);
  const int32_t *nf = categorical ? (h->ext_norm ? h->ext_norm : h->norm_flag) : nullptr;
  if (h->flags & LZM_TREE_EZ) hipLaunchKernelGGL(decode_backprop_kernel<true>, g, b, 0, s, p, nf);
  else hipLaunchKernelGGL(decode_backprop_kernel<false>, g, b, 0, s, p, nf);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_decode_backprop_traverse(lzm_handle *h, int cur, float discount, float *minmax, const float *reward_logits,
                                 const float *value_logits, int support_len, int categorical,
                                 const float *policy_logits, const int32_t *to_play, int lstm_horizon,
                                 int32_t *out_is_reset, const float *next_latent, float *pool_slot, int64_t row_elems,
                                 float *out_decoded, int pb_c_base, float pb_c_init, const uint32_t *seed,
                                 const int32_t *vtp_in, int32_t *out_x, int32_t *out_y, int32_t *out_a,
                                 int64_t *out_a64, int32_t *out_vtp, int32_t *out_len, void *stream) {
  if (!h || !minmax || !reward_logits || !value_logits || !policy_logits || !to_play || support_len <= 0 || !seed ||
      !vtp_in || !out_x || !out_y || !out_a || !out_vtp || !out_len) {
    set_err("lzm_decode_backprop_traverse: null argument");
    return LZM_ERR_ARG;
  }
  if (categorical && support_len % 2 == 0) {
    set_err("lzm_decode_backprop_traverse: categorical support length must be odd (2*support_scale+1)");
    return LZM_ERR_ARG;
  }
  if (pb_c_base <= 0) {
    set_err("lzm_decode_backprop_traverse: pb_c_base must be positive");
    return LZM_ERR_ARG;
  }
  if (h->flags & LZM_RNG_FAST) {
    set_err("lzm_decode_backprop_traverse: parity (glibc) mode only; use lzm_decode_backprop + lzm_traverse");
    return LZM_ERR_ARG;
  }
  int rc = check_cur(h, cur);
  if (rc != LZM_OK) return rc;
  rc = fill_lut(h, pb_c_base, pb_c_init);
  if (rc != LZM_OK) return rc;
  rc = ensure_coef(h, h->B * h->depth_cap + 64);
  if (rc != LZM_OK) return rc;
  rc = ensure_flags(h, 1, 1);
  if (rc != LZM_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (categorical && !h->ext_norm) {
    rc = launch_norm_check(h, h->norm_flag, reward_logits, value_logits, h->B, support_len, s);
    if (rc != LZM_OK) return rc;
  }
  DecodeArgs p;
  p.t = view(h);
  p.minmax = (float4 *)minmax;
  p.reward_logits = reward_logits; p.value_logits = value_logits; p.policy_logits = policy_logits;
  p.to_play = to_play; p.out_is_reset = out_is_reset; p.next_latent = next_latent; p.pool_slot = pool_slot;
  p.row_elems = row_elems; p.V = support_len; p.categorical = categorical; p.cur = cur; p.horizon = lstm_horizon;
  p.disc = discount; p.out_decoded = out_decoded;
  p.reuse_action = h->reuse_action; p.reuse_value = h->reuse_value;
  TraverseLbArgs q;
  q.t = p.t; q.minmax = (const float4 *)minmax; q.seed = seed; q.vtp_in = vtp_in;
  q.out_x = out_x; q.out_y = out_y; q.out_a = out_a; q.out_vtp = out_vtp; q.out_len = out_len;
  q.out_a64 = (long long *)out_a64; q.disc = discount;
  q.coef = h->coef; q.coef_positions = h->coef_positions; q.pow16807 = h->pow16807;
  q.flags = h->lb_flags; q.epoch = h->epoch; q.diag = h->diag; q.err = h->err;
  q.reuse_action = h->reuse_action; q.reuse_value = h->reuse_value;
  q.stamps = nullptr;
  const int per = kTlbThreads / 64;
  dim3 g((h->B + per - 1) / per), b(kTlbThreads);
  const int32_t *nf = categorical ? (h->ext_norm ? h->ext_norm : h->norm_flag) : nullptr;
  if (h->flags & LZM_TREE_EZ) hipLaunchKernelGGL(decode_traverse_kernel<true>, g, b, 0, s, p, nf, q);
  else hipLaunchKernelGGL(decode_traverse_kernel<false>, g, b, 0, s, p, nf, q);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static int32_t *g_scratch_flag = nullptr;
static int g_scratch_parts = 0;
static uint32_t *g_debug_jm = nullptr;  // lzm_debug_glibc_rand's jump matrices
static std::mutex g_scratch_mu;

int lzm_inverse_scalar_transform(const float *logits, int rows, int V, int categorical, float *out, void *stream) {
  if (!logits || !out || rows <= 0 || V <= 0) return LZM_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (g_scratch_parts < norm_parts(rows)) {
      // (grows only outside graph capture in practice: the first call sizes it)
      if (g_scratch_flag) LZM_HIP(hipFree(g_scratch_flag));
      g_scratch_flag = nullptr;
      LZM_HIP(hipMalloc(&g_scratch_flag, sizeof(int32_t) * 2 * norm_parts(rows)));
      g_scratch_parts = norm_parts(rows);
    }
  }
  if (categorical)
    hipLaunchKernelGGL(normalized_check_kernel, dim3(norm_parts(rows)), dim3(256), 0, s, logits, logits, rows, V,
                       g_scratch_flag);
  hipLaunchKernelGGL(inverse_transform_kernel, dim3((rows * 64 + 255) / 256), dim3(256), 0, s, logits, rows, V,
                     categorical, g_scratch_flag, out);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_get_distributions(lzm_handle *h, int32_t *out, void *stream) {
  if (!h || !out) return LZM_ERR_ARG;
  hipLaunchKernelGGL(distributions_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, view(h), out);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_get_values(lzm_handle *h, float *out, void *stream) {
  if (!h || !out) return LZM_ERR_ARG;
  hipLaunchKernelGGL(values_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, view(h), out);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_get_trajectories(lzm_handle *h, int32_t *out, int tmax, void *stream) {
  if (!h || !out || tmax <= 0) return LZM_ERR_ARG;
  hipLaunchKernelGGL(trajectories_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, view(h), out,
                     tmax);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_last_traverse_passes(lzm_handle *h, int32_t *out, void *stream) {
  if (!h || !out) return LZM_ERR_ARG;
  LZM_HIP(hipMemcpyAsync(out, h->diag, sizeof(int32_t) * 2, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return LZM_OK;
}

int lzm_debug_expf(const float *x, float *out, int64_t n, void *stream) {
  if (!x || !out || n <= 0) return LZM_ERR_ARG;
  long long grid = (n + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(debug_expf_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, x, out, (long long)n);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_debug_philox(const uint32_t *ck, uint32_t *out, int n, void *stream) {
  if (!ck || !out || n <= 0) return LZM_ERR_ARG;
  hipLaunchKernelGGL(debug_philox_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, ck, out, n);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// Process teardown (lightzero_amd registers it with atexit, before the interpreter finalises): wait for the
// device, then free the library's process-wide device buffers while the HIP runtime (and a profiler's
// hooks) are still in place, instead of leaving them to the runtime's own exit-time teardown. Live handles
// are destroyed by their owners first (lzm_destroy).
int lzm_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  LZM_HIP(hipDeviceSynchronize());
  if (g_scratch_flag) LZM_HIP(hipFree(g_scratch_flag));
  g_scratch_flag = nullptr;
  g_scratch_parts = 0;
  if (g_debug_jm) LZM_HIP(hipFree(g_debug_jm));
  g_debug_jm = nullptr;
  return LZM_OK;
}

int lzm_debug_az_rules(int n, const int32_t *boards, const double *scores, int32_t *out, void *stream) {
  if (n <= 0 || !boards || !scores || !out) return LZM_ERR_ARG;
  hipLaunchKernelGGL(debug_az_rules_kernel, dim3((n + 3) / 4), dim3(64), 0, (hipStream_t)stream, n, boards, scores, out);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_debug_xor(const float *in, float *out, void *stream) {
  if (!in || !out) return LZM_ERR_ARG;
  hipLaunchKernelGGL(debug_xor_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, in, out);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_debug_glibc_rand(uint32_t seed, int n, int32_t *out, void *stream) {
  if (!out || n <= 0) return LZM_ERR_ARG;
  uint32_t *&jm = g_debug_jm;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (!jm) {
      std::vector<uint32_t> jf, jn;
      build_jump_matrices(jf, jn);
      LZM_HIP(hipMalloc(&jm, sizeof(uint32_t) * 2 * kMaxWG * 31));
      LZM_HIP(hipMemcpy(jm, jf.data(), sizeof(uint32_t) * kMaxWG * 31, hipMemcpyHostToDevice));
      LZM_HIP(hipMemcpy(jm + kMaxWG * 31, jn.data(), sizeof(uint32_t) * kMaxWG * 31, hipMemcpyHostToDevice));
    }
  }
  hipLaunchKernelGGL(debug_glibc_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, seed, n, out, jm, jm + kMaxWG * 31);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- fused whole-search (MLP)
namespace {

// Layer shapes of the packed MuZeroModelMLP recurrent network (lzm_search_mlp.h order): krows
// input rows in the packed (torch-transposed) layout, K = krows rounded up to kKC in the kernel's.
struct LayerShape {
  int krows, K, N;
};
bool layer_used(int l, int res_dynamics) { return res_dynamics || (l != 2 && l != 3); }

// Kernel layers: the packed layers as the search kernel runs them. Two pairs are merged, each
// into one layer with columns [src0 | src1] over the same K: the value and policy head hiddens
// (fc_value_head[0] | fc_policy_head[0], same input) and the value and policy head outputs
// (fc_value_head[1] | fc_policy_head[1], inputs the two halves of that merged hidden) — fewer
// dependent steps per simulation, and fuller lanes.
struct KLayer {
  int src0, src1;  // packed layer indices (src1 < 0: single source)
  int K, N, N0;    // N0: columns taken from src0
};
int kernel_layers(const LayerShape *s, int res, KLayer *kl) {
  int n = 0;
  auto one = [&](int l) { kl[n++] = KLayer{l, -1, s[l].K, s[l].N, s[l].N}; };
  auto two = [&](int a, int b) { kl[n++] = KLayer{a, b, s[a].K, s[a].N + s[b].N, s[a].N}; };
  one(0);
  one(1);
  if (res) {
    one(2);
    one(3);
  }
  one(4);
  one(5);
  one(6);
  one(7);
  two(8, 10);
  two(9, 11);
  return n;
}
// float offsets of each packed layer (weights [krows][N], then bias [N]) in the packed buffer
void packed_offsets(const LayerShape *s, int res, size_t *w, size_t *b) {
  size_t off = 0;
  for (int l = 0; l < 12; ++l) {
    w[l] = b[l] = off;
    if (!layer_used(l, res)) continue;
    off += (size_t)s[l].krows * s[l].N;
    b[l] = off;
    off += s[l].N;
  }
}
// float offset of each kernel layer's weights / bias in the kernel layout (16-B aligned), total
size_t kernel_layout(const KLayer *kl, int nk, size_t *w_off, size_t *b_off) {
  size_t off = 0;
  for (int l = 0; l < nk; ++l) {
    w_off[l] = off;
    off += swz_floats(kl[l].K, kl[l].N);
    b_off[l] = off;
    off = (off + kl[l].N + 3) & ~(size_t)3;
  }
  return off;
}

// kernel-layout float d <- packed (k, col): col < N0 from src0 [krows0][N0], else src1 [krows1][N - N0]
__global__ void mlp_swizzle_kernel(const float *src0, int krows0, const float *src1, int krows1, int K, int N, int N0,
                                   float *dst, size_t n) {
  const size_t d = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  int k, col;
  swz_source(K, N, d, &k, &col);
  float v = 0.0f;
  if (col < N0) {
    if (k < krows0) v = src0[(size_t)k * N0 + col];
  } else if (col < N) {
    if (k < krows1) v = src1[(size_t)k * (N - N0) + (col - N0)];
  }
  dst[d] = v;
}
void mlp_shapes(int H, int A, int F, int V, LayerShape *s) {
  s[0] = {H + A, (H + A + kKC - 1) / kKC * kKC, H};  // fc_dynamics(_1)[0]: [latent; one-hot action]
  s[1] = {H, H, H};
  s[2] = {H, H, H};      // fc_dynamics_2 (res_connection_in_dynamics)
  s[3] = {H, H, H};
  s[4] = {H, H, F};      // fc_reward_head
  s[5] = {F, F, V};
  s[6] = {H, H, H};      // fc_prediction_common
  s[7] = {H, H, H};
  s[8] = {H, H, F};      // fc_value_head
  s[9] = {F, F, V};
  s[10] = {H, H, F};     // fc_policy_head
  s[11] = {F, F, A};
}

// Coefficients of z[344 + p] (the p-th rand() output before >> 1) over the 31 seeded words.
int ensure_coef(lzm_handle *h, int positions) {
  if (h->coef_positions >= positions) return LZM_OK;
  std::vector<uint32_t> tab((size_t)positions * 31);
  std::vector<uint32_t> ring((size_t)34 * 31, 0u);  // z[n] for n mod 34
  auto row = [&](long n) { return &ring[(size_t)(n % 34) * 31]; };
  for (int j = 0; j < 31; ++j) {
    uint32_t *r = row(j);
    for (int c = 0; c < 31; ++c) r[c] = (c == j);
  }
  for (int j = 31; j < 34; ++j) memcpy(row(j), row(j - 31), 31 * sizeof(uint32_t));
  const long last = 344L + positions;
  for (long n = 34; n < last; ++n) {
    uint32_t tmp[31];
    const uint32_t *a = row(n - 31), *b = row(n - 3);
    for (int c = 0; c < 31; ++c) tmp[c] = a[c] + b[c];
    memcpy(row(n), tmp, sizeof(tmp));
    if (n >= 344) memcpy(&tab[(size_t)(n - 344) * 31], tmp, sizeof(tmp));
  }
  dfree(h->coef);
  h->coef = nullptr;
  LZM_HIP(hipMalloc(&h->coef, tab.size() * sizeof(uint32_t)));
  LZM_HIP(hipMemcpy(h->coef, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  h->coef_positions = positions;
  if (!h->pow16807) {
    uint32_t pw[31];
    unsigned long long x = 1;
    for (int i = 0; i < 31; ++i) {
      pw[i] = (uint32_t)x;
      x = (x * 16807ull) % 2147483647ull;
    }
    LZM_HIP(hipMalloc(&h->pow16807, sizeof(pw)));
    LZM_HIP(hipMemcpy(h->pow16807, pw, sizeof(pw), hipMemcpyHostToDevice));
  }
  return LZM_OK;
}

int ensure_flags(lzm_handle *h, int sims, int G) {
  if (!h->epoch) {
    LZM_HIP(hipMalloc(&h->epoch, 2 * sizeof(uint32_t)));
    const uint32_t init[2] = {1u, 0u};
    LZM_HIP(hipMemcpy(h->epoch, init, sizeof(init), hipMemcpyHostToDevice));
    LZM_HIP(hipMalloc(&h->search_diag, 4 * sizeof(int32_t)));
    LZM_HIP(hipMemset(h->search_diag, 0, 4 * sizeof(int32_t)));
  }
  if (h->flag_sims >= sims) return LZM_OK;
  dfree(h->lb_flags);
  h->lb_flags = nullptr;
  const size_t n = (size_t)sims * std::max(G, h->B);  // any roots-per-workgroup choice fits
  LZM_HIP(hipMalloc(&h->lb_flags, n * sizeof(unsigned long long)));
  LZM_HIP(hipMemset(h->lb_flags, 0, n * sizeof(unsigned long long)));  // epoch 0 never matches
  h->flag_sims = sims;
  return LZM_OK;
}

// Roots per workgroup in the fused search: the smallest of 1, 2, 4, 8 that keeps the grid within
// one workgroup per CU (each simulation is a latency chain per workgroup, so spreading the batch
// over more CUs shortens it; fewer, fuller workgroups amortise each weight read over more rows).
// LZM_ROOTS_PER_WG overrides (experiments).
int roots_per_wg(int B) {
  const char *e = getenv("LZM_ROOTS_PER_WG");
  if (e) {
    const int r = atoi(e);
    if (r == 1 || r == 2 || r == 4 || r == 8) return r;
  }
  const int cus = device_cus();
  for (int r = 1; r < 8; r *= 2)
    if ((B + r - 1) / r <= cus) return r;
  return 8;
}

template <int R, bool TL>
hipError_t launch_search(const SearchArgs &p, int G, size_t lds, hipStream_t stream) {
  hipError_t e = hipFuncSetAttribute((const void *)search_mlp_kernel<R, TL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((search_mlp_kernel<R, TL>), dim3(G), dim3(kThreads), lds, stream, p);
  return hipGetLastError();
}

template <int R>
hipError_t launch_search_r(const SearchArgs &p, int G, size_t lds, hipStream_t stream) {
  return p.tree_in_lds ? launch_search<R, true>(p, G, lds, stream) : launch_search<R, false>(p, G, lds, stream);
}
constexpr size_t kMaxLds = 160 * 1024 - 1024;

size_t round4(size_t x) { return (x + 3) & ~(size_t)3; }

// The recurrent network as a schedule of dense steps over the kernel layers (LDS activation
// buffers by float offset): fc_dynamics(_1) on [latent; one-hot] (+ latent residual),
// fc_dynamics_2, reward head (decoded), fc_prediction_common, [value | policy] head hidden,
// [value | policy] head output: value decoded, policy logits [r][A] into X1
// (muzero_model_mlp.py:179-204, :420-440). Even length (two weight-prefetch buffers alternate).
void build_schedule(SearchArgs &p, const KLayer *kl, int nk, const size_t *w_off, const size_t *b_off,
                    const float *weights, int res, int A, int V, int F, int R) {
  const int x0 = (int)p.off_x0, x1 = (int)p.off_x1, x2 = (int)p.off_x2, nl = (int)p.off_n, hd = (int)p.off_h,
            lg = (int)p.off_logit;
  int n = 0, l = 0;
  auto add = [&](int in, int out, int relu, int resid, int rowmajor, int ldout, int dec) -> StepRec & {
    const KLayer &k = kl[l];
    StepRec &q = p.sched[n++];
    q.w = weights + w_off[l];
    q.b = weights + b_off[l];
    q.K = k.K;
    q.N = k.N;
    q.wbytes = (int)(swz_floats(k.K, k.N) * sizeof(float));
    q.in = in; q.out = out; q.relu = relu; q.resid = resid; q.rowmajor = rowmajor; q.ldout = ldout; q.decode = dec;
    q.ncol1 = k.N;  // columns routed like the first source (all, unless set below)
    q.in2 = in; q.out2 = out; q.rowmajor2 = rowmajor; q.ldout2 = ldout;
    const Split sp = layer_split(k.K, k.N);
    q.Np = sp.Np; q.splits = sp.splits; q.cpl = sp.cpl; q.log2s = sp.log2s;
    ++l;
    return q;
  };
  add(x0, x1, 1, -1, 0, 0, 0);                  // fc_dynamics(_1)[0]
  add(x1, nl, 1, res ? x0 : -1, 0, 0, 0);       // [1] (+ latent: res_connection_in_dynamics)
  int enc = nl;
  if (res) {
    add(nl, x1, 1, -1, 0, 0, 0);                // fc_dynamics_2
    add(x1, x2, 1, -1, 0, 0, 0);
    enc = x2;
  }
  p.stamp_at[0] = n - 1;
  add(enc, hd, 1, -1, 0, 0, 0);                 // fc_reward_head
  add(hd, lg, 0, -1, 1, V + 1, 1);
  p.stamp_at[1] = n - 1;
  add(nl, x1, 1, -1, 0, 0, 0);                  // fc_prediction_common
  add(x1, x2, 1, -1, 0, 0, 0);
  p.stamp_at[2] = n - 1;
  add(x2, hd, 1, -1, 0, 0, 0);                  // [fc_value_head[0] | fc_policy_head[0]]: 2F rows of hd
  StepRec &o = add(hd, lg, 0, -1, 1, V + 1, 2);  // [fc_value_head[1] | fc_policy_head[1]]
  o.ncol1 = V;                                  // value support columns, decoded
  o.in2 = hd + F / kKC * (kKC * R + 4);         // policy columns read the policy half of hd
  o.out2 = x1; o.rowmajor2 = 1; o.ldout2 = A;   // logits [r][A]
  p.stamp_at[3] = n - 1;
  p.nsteps = n;
  (void)nk;
}
// ---- network-resident search (lzm_search_res.h): the config-2 shape, one root per workgroup
bool res_shape_ok(int H, int A, int F, int V, int res) {
  return H == kRHid && F == kRF && V == kRV && res && A >= 1 && A <= kRMaxA;
}
bool res_enabled() {
  const char *e = getenv("LZM_FUSED_RES");  // "0": always the streaming kernel (experiments)
  return !(e && atoi(e) == 0);
}
struct ResSrc {
  size_t pw[12], pb[12];
  int N[12];
};
// resident float d <- packed network (res_source defines the layout)
__global__ void mlp_res_swizzle_kernel(const float *packed, ResSrc src, int A, float *dst, size_t n) {
  const size_t d = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  int b = 0;
  size_t o = 0;
  while (b + 1 < kRbN && d >= o + res_block_floats(b, A)) o += res_block_floats(b++, A);
  int layer, k, col;
  res_source(b, d - o, A, &layer, &k, &col);
  float v = 0.0f;
  if (layer >= 0) v = k < 0 ? packed[src.pb[layer] + col] : packed[src.pw[layer] + (size_t)k * src.N[layer] + col];
  dst[d] = v;
}
// LDS plan of search_res_kernel (float offsets, 16-B aligned); returns bytes, or 0 if it does not fit
size_t plan_res(SearchArgs &p, ResNet &n, const lzm_handle *h, int S, int A) {
  const ResPlan q = res_plan(h->cap, h->lut_n, h->depth_cap, S, A);
  n.plan = q;
  p.tree_in_lds = 1;
  p.off_stat = q.stat; p.off_meta = q.meta; p.off_lut = q.lut; p.off_legal = q.legal; p.off_val = q.val;
  p.off_path = q.path; p.off_pact = q.pact; p.off_misc = q.misc; p.off_pbt = q.pbt;
  p.pbt_rows = q.pbt_rows;
  return (size_t)q.floats * sizeof(float) <= (size_t)kResMaxBytes ? (size_t)q.floats * sizeof(float) : 0;
}
void res_net(ResNet &n, const float *wres, int A) {
  (void)A;
  n.w = wres;
}
}  // namespace

extern "C" {

int64_t lzm_mlp_packed_floats(int hidden, int actions, int head_hidden, int support, int res_dynamics) {
  if (hidden <= 0 || actions <= 0 || head_hidden <= 0 || support <= 0) return -1;
  LayerShape s[12];
  mlp_shapes(hidden, actions, head_hidden, support, s);
  int64_t n = 0;
  for (int l = 0; l < 12; ++l) {
    if (!res_dynamics && (l == 2 || l == 3)) continue;
    n += (int64_t)s[l].krows * s[l].N + s[l].N;
  }
  return n;
}

int64_t lzm_mlp_kernel_floats(int hidden, int actions, int head_hidden, int support, int res_dynamics) {
  if (hidden <= 0 || actions <= 0 || head_hidden <= 0 || support <= 0) return -1;
  LayerShape s[12];
  mlp_shapes(hidden, actions, head_hidden, support, s);
  KLayer kl[12];
  const int nk = kernel_layers(s, res_dynamics, kl);
  size_t w_off[12], b_off[12];
  size_t total = kernel_layout(kl, nk, w_off, b_off);
  // the network-resident kernel's layout follows (lzm_search_res.h), for the shape it serves
  if (res_shape_ok(hidden, actions, head_hidden, support, res_dynamics)) total = round4(total) + res_block_offset(kRbN, actions);
  return (int64_t)total;
}

int lzm_mlp_prepare(int hidden, int actions, int head_hidden, int support, int res_dynamics, const float *packed,
                    float *out, void *stream) {
  if (!packed || !out || hidden <= 0 || actions <= 0 || head_hidden <= 0 || support <= 0 ||
      hidden % kKC != 0 || head_hidden % kKC != 0) {
    set_err("lzm_mlp_prepare: bad arguments (hidden and head widths must be multiples of 16)");
    return LZM_ERR_ARG;
  }
  LayerShape s[12];
  mlp_shapes(hidden, actions, head_hidden, support, s);
  size_t pw[12], pb[12];
  packed_offsets(s, res_dynamics, pw, pb);
  KLayer kl[12];
  const int nk = kernel_layers(s, res_dynamics, kl);
  size_t w_off[12], b_off[12];
  kernel_layout(kl, nk, w_off, b_off);
  for (int l = 0; l < nk; ++l) {
    const KLayer &q = kl[l];
    const size_t n = swz_floats(q.K, q.N);
    const int s1 = q.src1 >= 0 ? q.src1 : q.src0;
    hipLaunchKernelGGL(mlp_swizzle_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       packed + pw[q.src0], s[q.src0].krows, packed + pw[s1], s[s1].krows, q.K, q.N, q.N0,
                       out + w_off[l], n);
    LZM_CHECK_LAUNCH();
    LZM_HIP(hipMemcpyAsync(out + b_off[l], packed + pb[q.src0], (size_t)q.N0 * sizeof(float),
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
    if (q.src1 >= 0)
      LZM_HIP(hipMemcpyAsync(out + b_off[l] + q.N0, packed + pb[q.src1], (size_t)(q.N - q.N0) * sizeof(float),
                             hipMemcpyDeviceToDevice, (hipStream_t)stream));
  }
  if (res_shape_ok(hidden, actions, head_hidden, support, res_dynamics)) {
    ResSrc src;
    for (int l = 0; l < 12; ++l) {
      src.pw[l] = pw[l];
      src.pb[l] = pb[l];
      src.N[l] = s[l].N;
    }
    const size_t base = round4(kernel_layout(kl, nk, w_off, b_off));
    const size_t n = res_block_offset(kRbN, actions);
    hipLaunchKernelGGL(mlp_res_swizzle_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       packed, src, actions, out + base, n);
    LZM_CHECK_LAUNCH();
  }
  return LZM_OK;
}

int lzm_search_mlp_kind(int B, int actions, int hidden, int head_hidden, int support, int res_dynamics) {
  if (B <= 0) return 0;
  return (roots_per_wg(B) == 1 && res_enabled() && res_shape_ok(hidden, actions, head_hidden, support, res_dynamics))
             ? 1
             : 0;
}

int lzm_search_mlp(lzm_handle *h, int hidden, int head_hidden, int support, int res_dynamics, const float *weights,
                   int num_simulations, int pb_c_base, float pb_c_init, float discount, float *minmax,
                   const uint32_t *seeds, const int32_t *vtp_in, float *latent_pool, int32_t *rec_x, int32_t *rec_a,
                   int32_t *rec_len, float *rec_decoded, float *rec_logits, void *stream) {
  if (!h || !weights || !minmax || (!seeds && !h->step_count) || !vtp_in || !latent_pool || num_simulations <= 0) {
    set_err("lzm_search_mlp: null argument or no simulations");
    return LZM_ERR_ARG;
  }
  if ((uintptr_t)weights & 15) {
    set_err("lzm_search_mlp: weights must be 16-byte aligned (lzm_mlp_prepare output)");
    return LZM_ERR_ARG;
  }
  if (h->flags & LZM_TREE_EZ) {
    set_err("lzm_search_mlp: MuZero trees only");
    return LZM_ERR_ARG;
  }
  const int H = hidden, F = head_hidden, V = support, A = h->A, S = num_simulations;
  if (H <= 0 || H > 1024 || F <= 0 || F > 1024 || V <= 0 || V + A > kMaxRounds * kThreads || A > H || H % kKC != 0 ||
      F % kKC != 0) {
    set_err("lzm_search_mlp: unsupported network shape (hidden and head widths must be multiples of 16)");
    return LZM_ERR_ARG;
  }
  if (S > h->sims_cap) {
    snprintf(g_err, sizeof(g_err), "lzm_search_mlp: %d simulations > reserved %d (lzm_reserve)", S, h->sims_cap);
    return LZM_ERR_CAPACITY;
  }
  int rc = fill_lut(h, pb_c_base, pb_c_init);
  if (rc != LZM_OK) return rc;
  const int R = roots_per_wg(h->B);
  const int G = (h->B + R - 1) / R;
  const bool fast = (h->flags & LZM_RNG_FAST) != 0;
  if (!fast) {
    rc = ensure_coef(h, h->B * (S + 1) + 64);
    if (rc != LZM_OK) return rc;
  }
  rc = ensure_flags(h, S, G);
  if (rc != LZM_OK) return rc;

  SearchArgs p;
  memset(&p, 0, sizeof(p));
  LayerShape shp[12];
  KLayer kls[12];
  int nkl = 0;
  size_t lay_w[12], lay_b[12];
  p.stat = h->stat; p.meta = h->meta; p.legal = h->legal; p.nlegal = h->nlegal;
  p.path = h->path; p.path_act = h->path_act; p.pathlen = h->pathlen; p.lut = h->lut;
  p.B = h->B; p.A = A; p.cap = h->cap; p.lut_n = h->lut_n; p.depth_cap = h->depth_cap;
  p.S = S; p.disc = discount; p.seeds = seeds; p.vtp_in = vtp_in; p.minmax = (float4 *)minmax; p.pool = latent_pool;
  p.H = H; p.F = F; p.V = V; p.res = res_dynamics ? 1 : 0;
  {
    LayerShape s[12];
    mlp_shapes(H, A, F, V, s);
    nkl = kernel_layers(s, res_dynamics, kls);
    kernel_layout(kls, nkl, lay_w, lay_b);
    for (int l = 0; l < 12; ++l) shp[l] = s[l];
  }
  p.coef = h->coef; p.coef_positions = h->coef_positions; p.pow16807 = h->pow16807;
  p.flags = h->lb_flags; p.epoch = h->epoch; p.diag = h->search_diag; p.fast = fast ? 1 : 0;
  if (!h->phase && getenv("LZM_PHASE_TIMING") && atoi(getenv("LZM_PHASE_TIMING")) > 0) {
    LZM_HIP(hipMalloc(&h->phase, (64 + 1024) * sizeof(unsigned long long)));
    LZM_HIP(hipMemset(h->phase, 0, (64 + 1024) * sizeof(unsigned long long)));
  }
  p.phase = h->phase;
  p.diag_mode = getenv("LZM_DIAG_MODE") ? atoi(getenv("LZM_DIAG_MODE")) : 0;  // timing experiments only
  p.rec_x = rec_x; p.rec_a = rec_a; p.rec_len = rec_len; p.rec_dec = rec_decoded; p.rec_logits = rec_logits;
  if (R == 1 && res_enabled() && res_shape_ok(H, A, F, V, res_dynamics)) {
    // the network-resident kernel (lzm_search_res.h); its weights follow the generic layout
    SearchArgs q = p;
    q.step_count = h->step_count; q.step_inc = h->step_inc; q.step_base = h->step_base; q.mm_fresh = h->step_fresh; q.mm_delta = h->step_delta;
    q.out_dist = h->step_dist; q.out_values = h->step_vals;
    ResNet n;
    memset(&n, 0, sizeof(n));
    const size_t lds = plan_res(q, n, h, S, A);
    if (lds) {
      res_net(n, weights + round4(kernel_layout(kls, nkl, lay_w, lay_b)), A);
      const char *sm = getenv("LZM_RES_SELECT");
      // measured: 4 < 1 < 0 < 2 < 3; 4 is 1 with the two-action walk for A == 2
      n.select_mode = sm ? atoi(sm) : (A == 2 ? 4 : 1);
      // LZM_RES_SPEC=1 (parity mode): evaluate two-way leaf ties speculatively as a second network
      // row instead of waiting for the look-back (measured slower: every simulation pays the row)
      const char *sl = getenv("LZM_RES_LATE");
      n.late_draw = sl ? atoi(sl) : 1;
      const char *sd = getenv("LZM_RES_SPEC_DEPTH");
      n.spec_depth = sd ? atoi(sd) : 1;
      const char *se = getenv("LZM_RES_SPEC");
      const bool spec = !fast && se && atoi(se) == 1;
      // production: selection mode, RNG and stamps fixed at compile time (modes 1 and 4); phase
      // timing compiles the stamps in; the other selection modes (experiments) read it at run time
      const int md = (n.select_mode == 4 && A != 2) ? 1 : n.select_mode;
      void (*fn)(SearchArgs, ResNet) =
          spec                  ? search_res_kernel<2, 1, 0, false>
          : (md != 1 && md != 4) || !n.spec_depth ? search_res_kernel<1, -1, -1, true>
          : q.phase             ? (md == 4 ? search_res_kernel<1, 4, -1, true> : search_res_kernel<1, 1, -1, true>)
          : md == 4             ? (fast ? search_res_kernel<1, 4, 1, false> : search_res_kernel<1, 4, 0, false>)
                                : (fast ? search_res_kernel<1, 1, 1, false> : search_res_kernel<1, 1, 0, false>);
      hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(fn, dim3(G), dim3(kRT), lds, (hipStream_t)stream, q, n);
        e = hipGetLastError();
      }
      LZM_HIP(e);
      LZM_CHECK_LAUNCH();
      return LZM_OK;
    }
  }
  // dynamic LDS plan (float offsets, 16-B aligned)
  size_t o = 0;
  const size_t tree_floats = (size_t)h->cap * R * 4;
  p.tree_in_lds = (2 * tree_floats * sizeof(float) <= 96 * 1024) ? 1 : 0;
  p.off_stat = o; if (p.tree_in_lds) o += tree_floats;
  p.off_meta = o; if (p.tree_in_lds) o += tree_floats;
  p.off_lut = o; if (p.tree_in_lds) o += round4((size_t)2 * h->lut_n);
  p.off_legal = o; if (p.tree_in_lds) o += round4((size_t)R * A + R);
  p.off_val = o; if (p.tree_in_lds) o += round4((size_t)h->cap * R);
  // pUCT visit table rows: all of lut when the triangle fits 32 KB (descent falls back to dividing)
  p.pbt_rows = (p.tree_in_lds && (size_t)h->lut_n * (h->lut_n + 1) / 2 <= 8192) ? h->lut_n : 0;
  p.off_pbt = o; o += round4((size_t)p.pbt_rows * (p.pbt_rows + 1) / 2);
  p.off_path = o; o += round4((size_t)h->depth_cap * R);
  p.off_pact = o; o += round4((size_t)h->depth_cap * R);
  // transposed activations [k][r], 4-float pad per kKC rows (tpos in lzm_search_mlp.h)
  auto tfl = [R](int K) { return (size_t)((K + kKC - 1) / kKC) * (kKC * R + 4); };
  p.off_x0 = o; o += round4(tfl(shp[0].K));  // [latent; one-hot] rows, zero-padded
  p.off_x1 = o; o += round4(tfl(H));          // also the policy logits [r][A]
  p.off_x2 = o; o += round4(tfl(H));
  p.off_n = o; o += round4(tfl(H));
  p.off_h = o; o += round4(tfl(2 * F));        // [value hidden; policy hidden] (merged layer)
  p.off_logit = o; if (V < kThreads) o += round4((size_t)(V + 1) * R);  // wide supports decode from registers
  p.off_part = o;  // (unused: split-K partials meet through DPP)
  p.off_misc = o; o += round4((size_t)S + 32);  // staged seeds[S] + 16807^i table
  const size_t lds = o * sizeof(float);
  build_schedule(p, kls, nkl, lay_w, lay_b, weights, res_dynamics, A, V, F, R);
  if (lds > kMaxLds) {
    snprintf(g_err, sizeof(g_err), "lzm_search_mlp: %zu B of LDS needed (network too wide)", lds);
    return LZM_ERR_ARG;
  }
  // collect-step mode: the prologue (seeds, fresh min-max) and epilogue (root outputs, counter)
  // as one launch each around the search
  if (h->step_count || h->step_fresh) {
    if (h->step_count && h->step_seeds_n < S) {  // (allocated with the tree: S <= sims_cap)
      set_err("lzm_search_mlp: step seeds buffer smaller than num_simulations (reserve first)");
      return LZM_ERR_STATE;
    }
    const int n = std::max(S, h->B);
    hipLaunchKernelGGL(step_prologue_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->step_count,
                       h->step_base, S, h->step_seeds, (float4 *)minmax, h->B, h->step_fresh, h->step_delta);
    LZM_CHECK_LAUNCH();
    if (h->step_count) p.seeds = reinterpret_cast<const uint32_t *>(h->step_seeds);
  }
  hipError_t e;
  switch (R) {
    case 1: e = launch_search_r<1>(p, G, lds, (hipStream_t)stream); break;
    case 2: e = launch_search_r<2>(p, G, lds, (hipStream_t)stream); break;
    case 4: e = launch_search_r<4>(p, G, lds, (hipStream_t)stream); break;
    default: e = launch_search_r<8>(p, G, lds, (hipStream_t)stream); break;
  }
  LZM_HIP(e);
  LZM_CHECK_LAUNCH();
  if ((h->step_count && h->step_inc) || h->step_dist || h->step_vals) {
    hipLaunchKernelGGL(step_epilogue_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, view(h),
                       h->step_dist, h->step_vals, h->step_inc ? h->step_count : nullptr);
    LZM_CHECK_LAUNCH();
  }
  return LZM_OK;
}

// Collect-step mode of lzm_search_mlp (sticky on the handle, host state only: a captured launch
// keeps the values it was launched with). See include/lzmcts.h.
int lzm_search_set_step(lzm_handle *h, int64_t *count, int64_t base, int increment, int32_t *root_dist,
                        float *root_values, int fresh_minmax, float value_delta_max) {
  if (!h || base < 0) return LZM_ERR_ARG;
  h->step_count = count;
  h->step_inc = increment ? 1 : 0;
  h->step_base = (long long)base;
  h->step_dist = root_dist;
  h->step_vals = root_values;
  h->step_fresh = fresh_minmax ? 1 : 0;
  h->step_delta = value_delta_max;
  return LZM_OK;
}

int lzm_debug_phase_cycles(lzm_handle *h, uint64_t *out_host, int reset) {
  if (!h || !out_host) return LZM_ERR_ARG;
  if (!h->phase) {
    memset(out_host, 0, 64 * sizeof(uint64_t));
    return LZM_OK;
  }
  LZM_HIP(hipDeviceSynchronize());
  LZM_HIP(hipMemcpy(out_host, h->phase, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (reset) LZM_HIP(hipMemset(h->phase, 0, 64 * sizeof(unsigned long long)));
  return LZM_OK;
}

// Diagnostics (LZM_PHASE_TIMING=1, resident kernel): shader-clock cycles each workgroup spent in
// the parity-mode look-back wait, summed over launches (phase[64 + g], up to 1024 workgroups).
int lzm_debug_root_wait_cycles(lzm_handle *h, uint64_t *out_host, int n, int reset) {
  if (!h || !out_host || n < 0 || n > 1024) return LZM_ERR_ARG;
  if (!h->phase) {
    memset(out_host, 0, n * sizeof(uint64_t));
    return LZM_OK;
  }
  LZM_HIP(hipDeviceSynchronize());
  LZM_HIP(hipMemcpy(out_host, h->phase + 64, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (reset) LZM_HIP(hipMemset(h->phase + 64, 0, 1024 * sizeof(unsigned long long)));
  return LZM_OK;
}

int lzm_search_diagnostics(lzm_handle *h, int32_t *out, void *stream) {
  if (!h || !out) return LZM_ERR_ARG;
  if (!h->search_diag) {
    LZM_HIP(hipMemsetAsync(out, 0, 4 * sizeof(int32_t), (hipStream_t)stream));
    return LZM_OK;
  }
  LZM_HIP(hipMemcpyAsync(out, h->search_diag, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return LZM_OK;
}

// Sticky error counters of every search path on this handle (a look-back spin that
// times out, or a draw position beyond the coefficient table, would otherwise leave a silently
// wrong tie-break stream; round 6: split-fp16 activations out of range). Synchronises `stream`;
// out_host (nullable) gets the kErrWords words {look-back timeouts, draw-table overflows, traverse
// fixed-point failures, fused-search errors, split-range errors, 0, 0, 0}.
int32_t *lzm_error_word(lzm_handle *h, int i) { return (h && i >= 0 && i < kErrWords) ? h->err + i : nullptr; }

int lzm_check_errors(lzm_handle *h, int32_t *out_host, int clear, void *stream) {
  if (!h) return LZM_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int32_t w[kErrWords] = {};
  int32_t sd = 0;
  LZM_HIP(hipMemcpyAsync(w, h->err, kErrWords * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (h->search_diag) LZM_HIP(hipMemcpyAsync(&sd, h->search_diag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  LZM_HIP(hipStreamSynchronize(s));
  w[3] += sd;  // err[3]: the EZ LSTM step's split-K hand-off timeouts (lzm_error_word(h, 3))
  if (out_host) memcpy(out_host, w, sizeof(w));
  const bool bad = w[0] || w[1] || w[2] || w[3] || w[4];
  if (bad && clear) {
    LZM_HIP(hipMemsetAsync(h->err, 0, kErrWords * sizeof(int32_t), s));
    if (h->search_diag) LZM_HIP(hipMemsetAsync(h->search_diag, 0, sizeof(int32_t), s));
    LZM_HIP(hipStreamSynchronize(s));
  }
  if (w[4]) {
    snprintf(g_err, sizeof(g_err),
             "split-fp16 network values out of range in %d workgroup-searches (non-finite, or beyond ~2^114): the "
             "search's network outputs are not f32-exact; run the conv network with precision='f32' "
             "(LZM_CONV_PRECISION=f32)", w[4]);
    return LZM_ERR_RANGE;
  }
  if (bad) {
    snprintf(g_err, sizeof(g_err),
             "search tie-break stream invalid: %d look-back timeouts, %d draw-table overflows, %d traverse "
             "fixed-point failures, %d fused-search errors (results differ from the reference)",
             w[0], w[1], w[2], w[3]);
    return LZM_ERR_STATE;
  }
  return LZM_OK;
}

int lzm_cartpole_reset(int n, double *state, int32_t *steps, float *obs, uint32_t seed, void *stream) {
  if (n <= 0 || !state || !steps || !obs) {
    set_err("lzm_cartpole_reset: bad arguments");
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(cartpole_reset_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, state,
                     steps, obs, seed);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_cartpole_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                              const float *pred_value, double *state, int32_t *steps, float *obs, float *noises,
                              float noise_alpha, float temperature, int deterministic, float *rec_obs,
                              int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                              float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                              uint32_t seed, const int64_t *counter, void *stream) {
  if (n <= 0 || A <= 0 || A > 64 || T <= 0 || E <= 0 || !visits || !root_value || !state || !steps || !obs ||
      !noises || !rec_obs || !rec_action || !rec_reward || !rec_visits || !rec_value || !ep_len || !ep_count ||
      !counter || !(temperature > 0.0f) || !(noise_alpha > 0.0f) || (!pred_value) != (!rec_pred)) {
    set_err("lzm_cartpole_collect_step: bad arguments");
    return LZM_ERR_ARG;
  }
  CollectArgs a;
  a.n = n; a.A = A; a.T = T; a.E = E; a.max_steps = max_steps; a.deterministic = deterministic;
  a.temperature = temperature; a.noise_alpha = noise_alpha; a.seed = seed; a.counter = counter;
  a.visits = visits; a.root_value = root_value; a.state = state; a.steps = steps; a.obs = obs; a.noises = noises;
  a.rec_obs = rec_obs; a.rec_action = rec_action; a.rec_reward = rec_reward; a.rec_visits = rec_visits;
  a.rec_value = rec_value; a.pred_value = pred_value; a.rec_pred = rec_pred; a.ep_len = ep_len;
  a.ep_count = ep_count; a.ep_return = ep_return;
  hipLaunchKernelGGL(cartpole_collect_kernel, dim3((n + 127) / 128), dim3(128), 0, (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static int atari_reset_g(int game, const char *name, int n, int32_t *state, int32_t *steps, uint8_t *cur, float *obs,
                         uint32_t seed, void *stream) {
  if (n <= 0 || !state || !steps || !cur || !obs || (((uintptr_t)cur | (uintptr_t)obs) & 15)) {
    snprintf(g_err, sizeof(g_err), "%s: bad arguments (16-B aligned frame buffers)", name);
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(game ? atari_reset_kernel<1> : atari_reset_kernel<0>, dim3(n), dim3(kAtThreads), 0,
                     (hipStream_t)stream, n, state, steps, cur, obs, seed);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static int atari_collect_step_g(int game, const char *name, int n, int A, int T, int E, const int32_t *visits,
                                const float *root_value, const float *pred_value, int32_t *state, int32_t *steps,
                                uint8_t *cur, float *obs, float *noises, float noise_alpha, float temperature,
                                int deterministic, uint8_t *rec_frames, int32_t *rec_action, float *rec_reward,
                                int32_t *rec_visits, float *rec_value, float *rec_pred, int32_t *ep_len,
                                int32_t *ep_count, float *ep_return, int max_steps, uint32_t seed,
                                const int64_t *counter, void *stream) {
  if (n <= 0 || A <= 0 || A > 64 || T <= 0 || E <= 0 || max_steps <= 0 || !visits || !root_value || !state || !steps ||
      !cur || !obs || !noises || !rec_frames || !rec_action || !rec_reward || !rec_visits || !rec_value || !ep_len ||
      !ep_count || !counter || !(temperature > 0.0f) || !(noise_alpha > 0.0f) || (!pred_value) != (!rec_pred) ||
      (((uintptr_t)cur | (uintptr_t)obs | (uintptr_t)rec_frames) & 15)) {
    snprintf(g_err, sizeof(g_err), "%s: bad arguments", name);
    return LZM_ERR_ARG;
  }
  AtariArgs a;
  a.n = n; a.A = A; a.T = T; a.E = E; a.max_steps = max_steps; a.deterministic = deterministic;
  a.temperature = temperature; a.noise_alpha = noise_alpha; a.seed = seed; a.counter = counter;
  a.visits = visits; a.root_value = root_value; a.state = state; a.steps = steps; a.cur = cur; a.obs = obs;
  a.noises = noises; a.rec_frames = rec_frames; a.rec_action = rec_action; a.rec_reward = rec_reward;
  a.rec_visits = rec_visits; a.rec_value = rec_value; a.pred_value = pred_value; a.rec_pred = rec_pred;
  a.ep_len = ep_len; a.ep_count = ep_count; a.ep_return = ep_return;
  hipLaunchKernelGGL(game ? atari_collect_kernel<1> : atari_collect_kernel<0>, dim3(n), dim3(kAtThreads), 0,
                     (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_atari_reset(int n, int32_t *state, int32_t *steps, uint8_t *cur, float *obs, uint32_t seed, void *stream) {
  return atari_reset_g(0, "lzm_atari_reset", n, state, steps, cur, obs, seed, stream);
}

int lzm_atari_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                           const float *pred_value, int32_t *state, int32_t *steps, uint8_t *cur, float *obs,
                           float *noises, float noise_alpha, float temperature, int deterministic, uint8_t *rec_frames,
                           int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                           float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                           uint32_t seed, const int64_t *counter, void *stream) {
  return atari_collect_step_g(0, "lzm_atari_collect_step", n, A, T, E, visits, root_value, pred_value, state, steps,
                              cur, obs, noises, noise_alpha, temperature, deterministic, rec_frames, rec_action,
                              rec_reward, rec_visits, rec_value, rec_pred, ep_len, ep_count, ep_return, max_steps, seed,
                              counter, stream);
}

int lzm_pong_reset(int n, int32_t *state, int32_t *steps, uint8_t *cur, float *obs, uint32_t seed, void *stream) {
  return atari_reset_g(1, "lzm_pong_reset", n, state, steps, cur, obs, seed, stream);
}

int lzm_pong_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                          const float *pred_value, int32_t *state, int32_t *steps, uint8_t *cur, float *obs,
                          float *noises, float noise_alpha, float temperature, int deterministic, uint8_t *rec_frames,
                          int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                          float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                          uint32_t seed, const int64_t *counter, void *stream) {
  return atari_collect_step_g(1, "lzm_pong_collect_step", n, A, T, E, visits, root_value, pred_value, state, steps,
                              cur, obs, noises, noise_alpha, temperature, deterministic, rec_frames, rec_action,
                              rec_reward, rec_visits, rec_value, rec_pred, ep_len, ep_count, ep_return, max_steps, seed,
                              counter, stream);
}

int lzm_episodes_scan(int n, int E, const int32_t *ep_count, const int32_t *consumed, const int32_t *ep_len,
                      int32_t *env_ep_off, int64_t *env_row_off, int64_t *totals, void *stream) {
  if (n <= 0 || E <= 0 || !ep_count || !consumed || !ep_len || !env_ep_off || !env_row_off || !totals) {
    set_err("lzm_episodes_scan: bad arguments");
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(episodes_scan_kernel, dim3(1), dim3(kTrScanThreads), 0, (hipStream_t)stream, n, E, ep_count,
                     consumed, ep_len, env_ep_off, env_row_off, totals);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// the conv representation network's per-convolution epilogue (include/lzmcts.h lzm_bias_add_relu):
// one float4 per thread, HBM-bound (one read of y (and z), one write)
__global__ __launch_bounds__(256) void bias_add_relu_kernel(float4 *__restrict__ y, const float *__restrict__ bias,
                                                            const float4 *__restrict__ z, int C, int HW4, long long n4,
                                                            int relu) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= n4) return;
  const float b = bias[(int)((q / HW4) % C)];
  float4 v = y[q];
  v.x += b; v.y += b; v.z += b; v.w += b;
  if (z) {
    const float4 r = z[q];
    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
  }
  if (relu) {
    v.x = fmaxf(v.x, 0.0f); v.y = fmaxf(v.y, 0.0f); v.z = fmaxf(v.z, 0.0f); v.w = fmaxf(v.w, 0.0f);
  }
  y[q] = v;
}

int lzm_bias_add_relu(float *y, const float *bias, const float *z, int N, int C, int HW, int relu, void *stream) {
  if (!y || !bias || N <= 0 || C <= 0 || HW <= 0 || HW % 4 || ((uintptr_t)y & 15) || ((uintptr_t)z & 15)) {
    set_err("lzm_bias_add_relu: bad arguments (HW % 4 == 0, 16-B aligned rows)");
    return LZM_ERR_ARG;
  }
  const long long n4 = (long long)N * C * (HW / 4);
  hipLaunchKernelGGL(bias_add_relu_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<float4 *>(y), bias, reinterpret_cast<const float4 *>(z), C, HW / 4, n4,
                     relu ? 1 : 0);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_episodes_pack(int n, int E, int T, int A, int has_pred, int64_t frame_bytes, const int32_t *ep_count,
                      const int32_t *ep_len, int32_t *consumed, const int32_t *env_ep_off, const int64_t *env_row_off,
                      const void *rec_frames, const int32_t *rec_action, const float *rec_reward,
                      const int32_t *rec_visits, const float *rec_value, const float *rec_pred,
                      const float *ep_return, void *out_frames, float *out_scalars, int64_t *out_index,
                      void *stream) {
  if (n <= 0 || E <= 0 || T <= 0 || A <= 0 || frame_bytes <= 0 || !ep_count || !ep_len || !consumed ||
      !env_ep_off || !env_row_off || !rec_frames || !rec_action || !rec_reward || !rec_visits || !rec_value ||
      (has_pred && !rec_pred) || !out_frames || !out_scalars || !out_index) {
    set_err("lzm_episodes_pack: bad arguments");
    return LZM_ERR_ARG;
  }
  PackArgs a;
  a.n = n; a.E = E; a.T = T; a.A = A; a.W = 3 + A + (has_pred ? 1 : 0); a.has_pred = has_pred ? 1 : 0;
  a.frame_bytes = frame_bytes; a.ep_count = ep_count; a.ep_len = ep_len; a.env_ep_off = env_ep_off;
  a.consumed = consumed; a.env_row_off = env_row_off;
  a.rec_frames = (const uint8_t *)rec_frames; a.rec_action = rec_action; a.rec_reward = rec_reward;
  a.rec_visits = rec_visits; a.rec_value = rec_value; a.rec_pred = rec_pred; a.ep_return = ep_return;
  a.out_frames = (uint8_t *)out_frames; a.out_scalars = out_scalars; a.out_index = out_index;
  if ((frame_bytes & 15) == 0 && (((uintptr_t)rec_frames | (uintptr_t)out_frames) & 15)) {
    set_err("lzm_episodes_pack: frame buffers must be 16-B aligned when frames are multiples of 16 B");
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(episodes_pack_kernel, dim3(n), dim3(kTrPackThreads), 0, (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

}  // extern "C"

// ---- batched AlphaZero (lzm_az.h). One workspace buffer per (B, S), carved here.
static int64_t az_carve(int B, int S, void *ws, AzTree *t) {
  const int64_t cap = 1 + (int64_t)kAzCells * (S + 1);
  char *p = (char *)ws;
  int64_t off = 0;
  auto take = [&](int64_t bytes) -> void * {
    void *r = p ? (void *)(p + off) : nullptr;
    off += (bytes + 255) & ~(int64_t)255;
    return r;
  };
  AzTree x;
  x.B = B; x.S = S; x.cap = (int)cap;
  const int64_t nodes = (int64_t)B * cap;
  x.visit = (int32_t *)take(nodes * 4);
  x.vsum = (float *)take(nodes * 4);
  x.prior = (float *)take(nodes * 4);
  x.first = (int32_t *)take(nodes * 4);
  x.nch = (int32_t *)take(nodes * 4);
  x.act = (int32_t *)take(nodes * 4);
  x.nnodes = (int32_t *)take((int64_t)B * 4);
  x.root_board = (int32_t *)take((int64_t)B * kAzCells * 4);
  x.root_player = (int32_t *)take((int64_t)B * 4);
  x.path = (int32_t *)take((int64_t)B * kAzPath * 4);
  x.leaf = (int32_t *)take((int64_t)B * 4 * 4);
  x.leaf_board = (int32_t *)take((int64_t)B * kAzCells * 4);
  x.lut_pb = (double *)take((int64_t)(S + 1) * 8);
  x.lut_sqrt = (double *)take((int64_t)(S + 1) * 8);
  x.noise = (double *)take((int64_t)kAzCells * kAzCells * 8);
  if (t) *t = x;
  return off;
}

static bool az_args_ok(int B, int S, const void *ws, const char *what) {
  if (B <= 0 || S <= 0 || S > (1 << 20) || !ws) {
    snprintf(g_err, sizeof(g_err), "%s: need B > 0, 0 < num_simulations <= 2^20 and a workspace", what);
    return false;
  }
  return true;
}

extern "C" {

int lzm_az_workspace_bytes(int B, int S, int64_t *out) {
  if (B <= 0 || S <= 0 || S > (1 << 20) || !out) {
    set_err("lzm_az_workspace_bytes: need B > 0, 0 < num_simulations <= 2^20");
    return LZM_ERR_ARG;
  }
  *out = az_carve(B, S, nullptr, nullptr);
  return LZM_OK;
}

int lzm_az_noise_table(double alpha, int max_n, double *out) {
  if (!(alpha > 0.0) || max_n <= 0 || max_n > 4096 || !out) {
    set_err("lzm_az_noise_table: need alpha > 0, 0 < max_n <= 4096");
    return LZM_ERR_ARG;
  }
  // _add_exploration_noise (mcts_alphazero.cpp:57-83): a default-seeded engine per call, so the
  // vector for n children is fixed: n gamma(alpha, 1) draws, each divided by their sum
  for (int n = 1; n <= max_n; ++n) {
    std::default_random_engine gen;
    std::gamma_distribution<double> dist(alpha, 1.0);
    std::vector<double> g((size_t)n);
    double sum = 0;
    for (int i = 0; i < n; ++i) {
      g[(size_t)i] = dist(gen);
      sum += g[(size_t)i];
    }
    for (int i = 0; i < max_n; ++i) out[(size_t)(n - 1) * max_n + i] = i < n ? g[(size_t)i] / sum : 0.0;
  }
  return LZM_OK;
}

int lzm_az_set_constants(int B, int S, void *ws, double pb_c_base, double pb_c_init, double alpha, void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_set_constants")) return LZM_ERR_ARG;
  if (!(pb_c_base > 0.0) || !(alpha > 0.0)) {
    set_err("lzm_az_set_constants: need pb_c_base > 0 and alpha > 0");
    return LZM_ERR_ARG;
  }
  AzTree t;
  az_carve(B, S, ws, &t);
  // _ucb_score (mcts_alphazero.cpp:47-54) over the integer parent count: glibc log / sqrt on the host
  std::vector<double> pb((size_t)S + 1), sq((size_t)S + 1), nz((size_t)kAzCells * kAzCells);
  for (int n = 0; n <= S; ++n) {
    pb[(size_t)n] = std::log((n + pb_c_base + 1) / pb_c_base) + pb_c_init;
    sq[(size_t)n] = std::sqrt((double)n);
  }
  lzm_az_noise_table(alpha, kAzCells, nz.data());
  hipStream_t s = (hipStream_t)stream;
  LZM_HIP(hipMemcpyAsync(t.lut_pb, pb.data(), pb.size() * 8, hipMemcpyHostToDevice, s));
  LZM_HIP(hipMemcpyAsync(t.lut_sqrt, sq.data(), sq.size() * 8, hipMemcpyHostToDevice, s));
  LZM_HIP(hipMemcpyAsync(t.noise, nz.data(), nz.size() * 8, hipMemcpyHostToDevice, s));
  LZM_HIP(hipStreamSynchronize(s));
  return LZM_OK;
}

int lzm_az_begin(int B, int S, void *ws, const int32_t *boards, const int32_t *start_index, float *state,
                 void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_begin")) return LZM_ERR_ARG;
  if (!boards || !start_index || !state) {
    set_err("lzm_az_begin: null buffer");
    return LZM_ERR_ARG;
  }
  AzTree t;
  az_carve(B, S, ws, &t);
  const int per = kAzThreads / kAzGroup;
  hipLaunchKernelGGL(az_begin_kernel, dim3((B + per - 1) / per), dim3(kAzThreads), 0, (hipStream_t)stream, t,
                     boards, start_index, state);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_az_step(int B, int S, void *ws, int sim, const float *probs, int pstride, const float *values, int vstride,
                int with_noise, double noise_weight, float *state, void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_step")) return LZM_ERR_ARG;
  if (sim < -1 || sim >= S || !probs || pstride < kAzCells || (sim >= 0 && (!values || vstride < 1)) || !state) {
    set_err("lzm_az_step: need -1 <= sim < num_simulations, probs [B][>=9], values [B] and a state buffer");
    return LZM_ERR_ARG;
  }
  AzTree t;
  az_carve(B, S, ws, &t);
  AzStepArgs a;
  a.sim = sim; a.with_noise = with_noise; a.noise_weight = noise_weight;
  a.probs = probs; a.pstride = pstride; a.values = values ? values : probs; a.vstride = vstride; a.state = state;
  const int per = kAzThreads / kAzGroup;
  hipLaunchKernelGGL(az_step_kernel, dim3((B + per - 1) / per), dim3(kAzThreads), 0, (hipStream_t)stream, t, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_az_finish(int B, int S, void *ws, double temperature, int sample, uint32_t seed, const int64_t *counter,
                  int32_t *visits, double *probs, int32_t *action, void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_finish")) return LZM_ERR_ARG;
  if (temperature == 0.0 || !visits || !probs || !action) {
    set_err("lzm_az_finish: temperature cannot be 0; visits / probs / action buffers required");
    return LZM_ERR_ARG;
  }
  AzTree t;
  az_carve(B, S, ws, &t);
  hipLaunchKernelGGL(az_finish_kernel, dim3((B + 127) / 128), dim3(128), 0, (hipStream_t)stream, t, temperature,
                     sample, seed, counter, visits, probs, action);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_az_export_tree(int B, int S, void *ws, int32_t *visit, float *vsum, int32_t *first, int32_t *nnodes,
                       void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_export_tree")) return LZM_ERR_ARG;
  AzTree t;
  az_carve(B, S, ws, &t);
  hipStream_t s = (hipStream_t)stream;
  const size_t nodes = (size_t)B * t.cap;
  if (visit) LZM_HIP(hipMemcpyAsync(visit, t.visit, nodes * 4, hipMemcpyDeviceToDevice, s));
  if (vsum) LZM_HIP(hipMemcpyAsync(vsum, t.vsum, nodes * 4, hipMemcpyDeviceToDevice, s));
  if (first) LZM_HIP(hipMemcpyAsync(first, t.first, nodes * 4, hipMemcpyDeviceToDevice, s));
  if (nnodes) LZM_HIP(hipMemcpyAsync(nnodes, t.nnodes, (size_t)B * 4, hipMemcpyDeviceToDevice, s));
  return LZM_OK;
}

}  // extern "C"

// ---- fused AlphaZero search (lzm_az_fused.h)
template <int R>
static size_t az_fused_lds(int cap, int S) {
  // the double tables padded to 16 B, the node records, the network (az_search_fused_kernel's carve)
  const size_t bytes = (size_t)((2 * (S + 1) + 81 + 1) & ~1) * 8 + (size_t)R * cap * 16 + 128;
  return bytes + (size_t)AzNetLds<R>::total * 4;
}

template <int R, int NRES>
static int az_fused_attr(bool stamps) {
  static bool attr[2] = {false, false};
  if (!attr[stamps]) {
    LZM_HIP(hipFuncSetAttribute(stamps ? (const void *)az_search_fused_kernel<R, NRES, true>
                                       : (const void *)az_search_fused_kernel<R, NRES, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr[stamps] = true;
  }
  return LZM_OK;
}

// workgroups of R boards that one CU holds at once (0: the trees do not fit in LDS)
template <int R, int NRES>
static int az_fused_per_cu(int cap, int S, bool stamps) {
  const size_t lds = az_fused_lds<R>(cap, S);
  if (lds > 160 * 1024) return 0;
  static size_t memo_lds[2] = {0, 0};
  static int memo[2] = {0, 0};
  if (memo_lds[stamps] == lds) return memo[stamps];
  if (az_fused_attr<R, NRES>(stamps) != LZM_OK) return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stamps ? (const void *)az_search_fused_kernel<R, NRES, true>
                                                                   : (const void *)az_search_fused_kernel<R, NRES, false>,
                                                   kAzfThreads, lds) != hipSuccess)
    per_cu = 1;
  memo_lds[stamps] = lds;
  memo[stamps] = per_cu;
  return per_cu;
}

// boards per workgroup: the fewest whose grid the GPU holds at once (B = 512 on 256 CUs: one board per
// workgroup, two workgroups per CU, so each CU interleaves two boards' latency chains); else the most that fit
template <int NRES>
static int az_fused_rows(int B, int cap, int S, bool stamps) {
  const char *e = getenv("LZM_AZ_BOARDS_PER_WG");
  if (e && atoi(e) > 0) return atoi(e);
  const int cus = device_cus();
  const int occ[4] = {az_fused_per_cu<1, NRES>(cap, S, stamps), az_fused_per_cu<2, NRES>(cap, S, stamps),
                      az_fused_per_cu<4, NRES>(cap, S, stamps), az_fused_per_cu<8, NRES>(cap, S, stamps)};
  int best = 0;
  for (int i = 0, r = 1; i < 4; ++i, r *= 2) {
    if (!occ[i]) continue;
    best = r;
    if ((B + r - 1) / r <= occ[i] * cus) return r;
  }
  return best ? best : 1;
}

template <int R, int NRES>
static int az_launch_fused(const AzFusedArgs &a, hipStream_t s) {
  const size_t lds = az_fused_lds<R>(a.cap, a.S);
  if (lds > 160 * 1024) {
    snprintf(g_err, sizeof(g_err), "lzm_az_search_fused: %d boards x %d simulations need %zu B of LDS per workgroup (> 160 KiB)",
             R, a.S, lds);
    return LZM_ERR_CAPACITY;
  }
  // diagnostics: lzm_debug_az_stamps selects the stamped instantiation
  if (int rc = az_fused_attr<R, NRES>(a.stamps != nullptr)) return rc;
  auto fn = a.stamps ? az_search_fused_kernel<R, NRES, true> : az_search_fused_kernel<R, NRES, false>;
  hipLaunchKernelGGL(fn, dim3((a.B + R - 1) / R), dim3(kAzfThreads), lds, s, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

template <int NRES>
static int az_launch_fused_r(int R, const AzFusedArgs &a, hipStream_t s) {
  switch (R) {
    case 1: return az_launch_fused<1, NRES>(a, s);
    case 2: return az_launch_fused<2, NRES>(a, s);
    case 4: return az_launch_fused<4, NRES>(a, s);
    case 8: return az_launch_fused<8, NRES>(a, s);
  }
  set_err("lzm_az_search_fused: boards per workgroup must be 1, 2, 4 or 8");
  return LZM_ERR_ARG;
}

template <int R, int NRES>
static int az_launch_eval(const float *w, const float *state, int n, float *probs, float *value, hipStream_t s) {
  const size_t lds = (size_t)AzNetLds<R>::total * 4;
  static bool attr = false;
  if (!attr) {
    LZM_HIP(hipFuncSetAttribute((const void *)az_net_eval_kernel<R, NRES>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((az_net_eval_kernel<R, NRES>), dim3((n + R - 1) / R), dim3(kAzfThreads), lds, s, w, state, n,
                     probs, value);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

static unsigned long long *g_az_stamps = nullptr;  // diagnostics: lzm_debug_az_stamps

extern "C" {

// Diagnostics: a device uint64[8] that the fused AlphaZero search adds its per-phase shader-clock cycles to
// (AzFusedArgs::stamps); nullptr returns to the production instantiation.
int lzm_debug_az_stamps(void *buf) {
  g_az_stamps = reinterpret_cast<unsigned long long *>(buf);
  return LZM_OK;
}

int64_t lzm_az_net_floats(int nres) { return nres == 1 || nres == 2 ? az_net_layout(nres).total : -1; }

int lzm_az_net_prepare(int nres, const float *raw, float *out) {
  if ((nres != 1 && nres != 2) || !raw || !out) {
    set_err("lzm_az_net_prepare: num_res_blocks must be 1 or 2");
    return LZM_ERR_ARG;
  }
  const AzNetLayout L = az_net_layout(nres);
  memset(out, 0, sizeof(float) * (size_t)L.total);
  const float *p = raw;
  const float *w0 = p; p += 16 * 27;
  const float *b0 = p; p += 16;
  for (int s = 0; s < 7; ++s)
    for (int lane = 0; lane < 64; ++lane) {
      const int k = 4 * s + (lane >> 4);
      out[L.conv0 + s * 64 + lane] = k < 27 ? w0[(lane & 15) * 27 + k] : 0.0f;
    }
  memcpy(out + L.conv0_b, b0, 16 * sizeof(float));
  for (int l = 0; l < 4 * nres; ++l) {
    const float *wl = p; p += 16 * 144;
    const float *bl = p; p += 16;
    for (int s = 0; s < 36; ++s)
      for (int lane = 0; lane < 64; ++lane)
        out[L.res + (l * 36 + s) * 64 + lane] = wl[(lane & 15) * 144 + 4 * s + (lane >> 4)];
    memcpy(out + L.res_b + l * 16, bl, 16 * sizeof(float));
  }
  const float *wh = p; p += 32 * 16;
  const float *bh = p; p += 32;
  for (int s = 0; s < 4; ++s)
    for (int nt = 0; nt < 2; ++nt)
      for (int lane = 0; lane < 64; ++lane)
        out[L.head + (s * 2 + nt) * 64 + lane] = wh[(16 * nt + (lane & 15)) * 16 + 4 * s + (lane >> 4)];
  memcpy(out + L.head_b, bh, 32 * sizeof(float));
  memcpy(out + L.heads, p, kAzHeadFloats * sizeof(float));
  return LZM_OK;
}

int lzm_az_net_eval(int nres, const float *weights, const float *state, int n, float *probs, float *value,
                    void *stream) {
  if ((nres != 1 && nres != 2) || !weights || !state || n <= 0 || !probs || !value) {
    set_err("lzm_az_net_eval: need num_res_blocks 1 or 2, n > 0 and all buffers");
    return LZM_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  return nres == 1 ? az_launch_eval<2, 1>(weights, state, n, probs, value, s)
                   : az_launch_eval<2, 2>(weights, state, n, probs, value, s);
}

int lzm_az_search_fused(int B, int S, void *ws, int nres, const float *weights, const int32_t *boards,
                        const int32_t *start_index, int with_noise, double noise_weight, double temperature,
                        int sample, uint32_t seed, const int64_t *counter, int32_t *visits, double *probs,
                        int32_t *action, int export_tree, void *stream) {
  if (!az_args_ok(B, S, ws, "lzm_az_search_fused")) return LZM_ERR_ARG;
  if ((nres != 1 && nres != 2) || !weights || !boards || !start_index || temperature == 0.0 || !visits || !probs ||
      !action) {
    set_err("lzm_az_search_fused: need num_res_blocks 1 or 2, temperature != 0 and all buffers");
    return LZM_ERR_ARG;
  }
  if (1 + kAzCells * (S + 1) >= 0xffff) {
    set_err("lzm_az_search_fused: num_simulations too large for the LDS tree (16-bit node index)");
    return LZM_ERR_CAPACITY;
  }
  AzFusedArgs a;
  az_carve(B, S, ws, &a.t);
  a.B = B; a.S = S; a.cap = a.t.cap; a.with_noise = with_noise; a.sample = sample; a.export_tree = export_tree;
  a.noise_weight = noise_weight; a.temperature = temperature; a.seed = seed; a.counter = counter; a.w = weights;
  a.boards = boards; a.start_index = start_index; a.visits_out = visits; a.probs_out = probs; a.action_out = action;
  a.stamps = g_az_stamps;
  const int R = nres == 1 ? az_fused_rows<1>(B, a.cap, S, a.stamps != nullptr) : az_fused_rows<2>(B, a.cap, S, a.stamps != nullptr);
  hipStream_t s = (hipStream_t)stream;
  return nres == 1 ? az_launch_fused_r<1>(R, a, s) : az_launch_fused_r<2>(R, a, s);
}


int64_t lzm_conv_trunk_floats_p(int n_dres, int n_pres, int precision) {
  if (n_dres < 0 || n_pres < 0 || n_dres > 8 || n_pres > 8 || (precision != LZM_CONV_F32 && precision != LZM_CONV_SPLIT))
    return -1;
  return conv_trunk_layout_p(n_dres, n_pres, precision).total;
}

int64_t lzm_conv_trunk_floats(int n_dres, int n_pres) { return lzm_conv_trunk_floats_p(n_dres, n_pres, LZM_CONV_F32); }

int lzm_conv_trunk_prepare_p(int precision, int n_dres, int n_pres, int r_ch, int h_ch, const float *raw, float *out) {
  if (lzm_conv_trunk_floats_p(n_dres, n_pres, precision) < 0 || r_ch < 1 || r_ch > 32 || h_ch < 1 || h_ch > 32 ||
      !raw || !out) {
    set_err("lzm_conv_trunk_prepare: need 0..8 residual blocks, 1..32 reward / head channels, a known precision and "
            "buffers");
    return LZM_ERR_ARG;
  }
  const bool bx = precision == LZM_CONV_SPLIT;
  const ConvTrunkLayout L = conv_trunk_layout_p(n_dres, n_pres, precision);
  const int frag3 = bx ? kBx3Frag : kCv3Frag, block = bx ? kBxBlock : kCvBlock;
  const int n3 = 1 + 2 * (n_dres + n_pres);
  // split: layer li's row scales at sc + 64 li, its bounds {Wb, Bb} at bd + 4 li (3x3 layers in order, then the
  // reward and head 1x1s); the dynamics conv's Bb (max |actmap|) is set by lzm_conv_trunk_actmap_bound
  auto pack3 = [&](const float *W, float *o, int li, const float *bias) {
    if (!bx) return conv_pack3(W, o);
    bx_pack3(W, o, out + L.sc + 64 * li, out + L.bd + 4 * li);
    out[L.bd + 4 * li + 1] = bias ? bx_bias_bound(bias, 64) : 0.f;
  };
  auto pack1 = [&](const float *W, int n, float *o, int li, const float *bias) {
    if (!bx) return conv_pack1(W, n, o);
    bx_pack1(W, n, o, out + L.sc + 64 * li, out + L.bd + 4 * li);
    out[L.bd + 4 * li + 1] = bx_bias_bound(bias, n);
  };
  memset(out, 0, sizeof(float) * (size_t)L.total);
  const float *r = raw;
  const int W3 = 64 * 64 * 9;
  pack3(r, out + L.dyn, 0, nullptr); r += W3;
  auto blocks = [&](int n, int base, int li0) {
    for (int k = 0; k < n; ++k) {
      float *o = out + base + k * block;
      pack3(r, o, li0 + 2 * k, r + W3); r += W3;
      memcpy(o + frag3, r, 64 * sizeof(float)); r += 64;
      pack3(r, o + frag3 + 64, li0 + 2 * k + 1, r + W3); r += W3;
      memcpy(o + 2 * frag3 + 64, r, 64 * sizeof(float)); r += 64;
    }
  };
  blocks(n_dres, L.dres, 1);
  pack1(r, r_ch, out + L.rw, n3, r + r_ch * 64); r += r_ch * 64;
  memcpy(out + L.rb, r, r_ch * sizeof(float)); r += r_ch;
  blocks(n_pres, L.pres, 1 + 2 * n_dres);
  pack1(r, h_ch, out + L.hw, n3 + 1, r + h_ch * 64); r += h_ch * 64;
  memcpy(out + L.hb, r, h_ch * sizeof(float));
  return LZM_OK;
}

int lzm_conv_trunk_actmap_bound(int n_dres, int n_pres, float actmap_absmax, float *packed) {
  if (lzm_conv_trunk_floats_p(n_dres, n_pres, LZM_CONV_SPLIT) < 0 || !packed || !(actmap_absmax >= 0.f)) {
    set_err("lzm_conv_trunk_actmap_bound: a split-layout blob and a finite max |actmap| >= 0");
    return LZM_ERR_ARG;
  }
  packed[conv_trunk_layout_p(n_dres, n_pres, LZM_CONV_SPLIT).bd + 1] = bx_round_up(actmap_absmax);
  return LZM_OK;
}

int lzm_conv_trunk_prepare(int n_dres, int n_pres, int r_ch, int h_ch, const float *raw, float *out) {
  return lzm_conv_trunk_prepare_p(LZM_CONV_F32, n_dres, n_pres, r_ch, h_ch, raw, out);
}

int lzm_conv_trunk_xin_p(int precision, int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights,
                         const float *actmap, const float *pool, const int32_t *x, const int32_t *action,
                         float *out_latent, float *xin, int xin_stride, const float *hpool, int H, int32_t *xscale,
                         float *out_h, int32_t *err, void *stream) {
  if (B <= 0 || lzm_conv_trunk_floats_p(n_dres, n_pres, precision) < 0 || r_ch < 1 || r_ch > 32 || h_ch < 1 ||
      h_ch > 32 || !weights || !actmap || !pool || !action || !out_latent || !xin || !out_h ||
      xin_stride < r_ch * 64 + (hpool ? H : 0) || (hpool && (H <= 0 || H % 4)) || xin_stride % 4) {
    set_err("lzm_conv_trunk: bad arguments");
    return LZM_ERR_ARG;
  }
  if (((uintptr_t)weights | (uintptr_t)pool | (uintptr_t)xin | (uintptr_t)hpool) & 15) {
    set_err("lzm_conv_trunk: weights, pool, xin and hpool must be 16-byte aligned");
    return LZM_ERR_ARG;
  }
  float *out_r = xin;
  const bool bx = precision == LZM_CONV_SPLIT;
  static std::once_flag once;
  static hipError_t attr_err = hipSuccess;
  const size_t lds_f32 = 3 * kCvBuf * sizeof(float), lds_bx = 2 * kBxBuf * sizeof(uint16_t);
  std::call_once(once, [&] {
    attr_err = hipFuncSetAttribute((const void *)conv_trunk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_f32);
    if (attr_err == hipSuccess)
      attr_err = hipFuncSetAttribute((const void *)conv_trunk_bx_kernel<kBxAhead>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bx);
  });
  LZM_HIP(attr_err);
  ConvTrunkArgs a;
  a.B = B; a.n_dres = n_dres; a.n_pres = n_pres; a.r_ch = r_ch; a.h_ch = h_ch; a.w = weights; a.actmap = actmap;
  a.pool = pool; a.x = x; a.action = action; a.out_latent = out_latent; a.out_r = out_r; a.out_h = out_h;
  a.r_stride = xin_stride; a.hpool = hpool; a.H = hpool ? H : 0; a.skip_dyn = 0; a.err = err;
  a.xscale = precision == LZM_CONV_SPLIT ? xscale : nullptr;
  if (bx)
    hipLaunchKernelGGL(conv_trunk_bx_kernel<kBxAhead>, dim3(B), dim3(kCvThreads), lds_bx, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(conv_trunk_kernel, dim3(B), dim3(kCvThreads), lds_f32, (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_conv_trunk_p(int precision, int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights,
                     const float *actmap, const float *pool, const int32_t *x, const int32_t *action, float *out_latent,
                     float *out_r, float *out_h, int32_t *err, void *stream) {
  return lzm_conv_trunk_xin_p(precision, B, n_dres, n_pres, r_ch, h_ch, weights, actmap, pool, x, action, out_latent,
                              out_r, r_ch * 64, nullptr, 0, nullptr, out_h, err, stream);
}

int lzm_conv_resnet8_p(int B, int n_blocks, int n_pres, int h_ch, const float *weights, const float *in,
                       float *out_latent, float *out_h, int32_t *err, void *stream) {
  if (B <= 0 || n_blocks < 1 || lzm_conv_trunk_floats_p(n_blocks, n_pres, LZM_CONV_SPLIT) < 0 || h_ch < 1 ||
      h_ch > 32 || !weights || !in || !out_latent || !out_h || (((uintptr_t)weights | (uintptr_t)in) & 15)) {
    set_err("lzm_conv_resnet8_p: bad arguments (1..8 blocks, 1..32 head channels, 16-byte aligned weights / input)");
    return LZM_ERR_ARG;
  }
  static hipError_t attr_err = hipFuncSetAttribute((const void *)conv_trunk_bx_kernel<kBxAhead>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)(2 * kBxBuf * sizeof(uint16_t)));
  LZM_HIP(attr_err);
  ConvTrunkArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.n_dres = n_blocks; a.n_pres = n_pres; a.r_ch = 0; a.h_ch = h_ch; a.w = weights;
  a.pool = in; a.out_latent = out_latent; a.out_h = out_h; a.skip_dyn = 1; a.err = err;
  hipLaunchKernelGGL((conv_trunk_bx_kernel<kBxAhead>), dim3(B), dim3(kCvThreads), 2 * kBxBuf * sizeof(uint16_t),
                     (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// ---- the representation network's DownSample stages (lzm_repr.h)
int64_t lzm_repr_floats(void) { return repr_layout().total; }

int lzm_repr_prepare(int cin, const float *raw, float *out) {
  if (cin < 1 || cin * 9 > 64 || !raw || !out) {
    set_err("lzm_repr_prepare: 1..7 observation channels and buffers");
    return LZM_ERR_ARG;
  }
  const ReprLayout L = repr_layout();
  memset(out, 0, sizeof(float) * (size_t)L.total);
  const float *r = raw;
  auto bias = [&](int off, int n) { memcpy(out + off, r, n * sizeof(float)); r += n; };
  repr_pack(r, 32, cin, true, out + L.w1, out + L.s1); r += 32 * cin * 9; bias(L.b1, 32);
  repr_pack(r, 32, 32, false, out + L.r1w1, out + L.r1s1); r += 32 * 32 * 9; bias(L.r1b1, 32);
  repr_pack(r, 32, 32, false, out + L.r1w2, out + L.r1s2); r += 32 * 32 * 9; bias(L.r1b2, 32);
  // the downsample block: conv1 (64) and the shortcut conv3 (64) stacked as one 128-channel layer
  std::vector<float> dual((size_t)128 * 32 * 9);
  memcpy(dual.data(), r, sizeof(float) * 64 * 32 * 9); r += 64 * 32 * 9;
  bias(L.db1, 64);
  const float *w2 = r; r += 64 * 64 * 9;
  bias(L.db2, 64);
  memcpy(dual.data() + 64 * 32 * 9, r, sizeof(float) * 64 * 32 * 9); r += 64 * 32 * 9;
  repr_pack(dual.data(), 128, 32, false, out + L.dw, out + L.ds);
  repr_pack(w2, 64, 64, false, out + L.dw2, out + L.ds2);
  repr_pack(r, 64, 64, false, out + L.r2w1, out + L.r2s1); r += 64 * 64 * 9; bias(L.r2b1, 64);
  repr_pack(r, 64, 64, false, out + L.r2w2, out + L.r2s2); r += 64 * 64 * 9; bias(L.r2b2, 64);
  return LZM_OK;
}

int64_t lzm_repr_workspace_floats(int B) { return B <= 0 ? -1 : (int64_t)B * (2 * 32 * 32 * 32 + 2 * 16 * 16 * 64); }

}  // extern "C"

template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
static int repr_launch(const ReprConvArgs &a, hipStream_t s) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE, RES> G;
  const size_t lds = G::LDSB;
  static hipError_t attr = hipFuncSetAttribute((const void *)repr_conv_kernel<CIN, COUT, STRIDE, WOUT, MODE, RES>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  LZM_HIP(attr);
  const int grid = std::min(a.ntiles, device_cus());
  hipLaunchKernelGGL((repr_conv_kernel<CIN, COUT, STRIDE, WOUT, MODE, RES>), dim3(grid), dim3(kRpThreads), lds, s, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" {

int lzm_repr_downsample(int B, int cin, const float *w, const float *obs, float *ws, float *out, void *stream) {
  if (B <= 0 || cin < 1 || cin * 9 > 64 || !w || !obs || !ws || !out ||
      (((uintptr_t)w | (uintptr_t)ws | (uintptr_t)out) & 15)) {
    set_err("lzm_repr_downsample: bad arguments (1..7 observation channels, 16-byte aligned weights / workspace)");
    return LZM_ERR_ARG;
  }
  const ReprLayout L = repr_layout();
  hipStream_t s = (hipStream_t)stream;
  float *A0 = ws, *A1 = ws + (size_t)B * 32768, *D0 = ws + (size_t)B * 65536, *D1 = D0 + (size_t)B * 16384;
  ReprConvArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.cin_obs = cin;
  int rc;
  // L1: obs (NCHW 64 x 64) -> A0 [32][32][32] (128-pixel tiles: 8 per image)
  a.ntiles = B * 8; a.in = obs; a.w = w + L.w1; a.winv = w + L.s1; a.bias = w + L.b1; a.res = nullptr; a.out = A0;
  if ((rc = repr_launch<32, 32, 2, 32, 2, false>(a, s)) != LZM_OK) return rc;
  // resblocks1: A0 -> A1 -> A0 (+ A0)
  a.in = A0; a.w = w + L.r1w1; a.winv = w + L.r1s1; a.bias = w + L.r1b1; a.out = A1;
  if ((rc = repr_launch<32, 32, 1, 32, 0, false>(a, s)) != LZM_OK) return rc;
  a.in = A1; a.w = w + L.r1w2; a.winv = w + L.r1s2; a.bias = w + L.r1b2; a.res = A0; a.out = A0;
  if ((rc = repr_launch<32, 32, 1, 32, 0, true>(a, s)) != LZM_OK) return rc;
  // the downsample block: A0 -> D0 = relu(conv1 + b1), D1 = conv3 (shortcut); D1 = relu(conv2(D0) + b2 + D1)
  a.ntiles = B * 4; a.in = A0; a.w = w + L.dw; a.winv = w + L.ds; a.bias = w + L.db1; a.res = nullptr; a.out = D0;
  a.out2 = D1;
  if ((rc = repr_launch<32, 128, 2, 16, 1, false>(a, s)) != LZM_OK) return rc;
  a.in = D0; a.w = w + L.dw2; a.winv = w + L.ds2; a.bias = w + L.db2; a.res = D1; a.out = D1; a.out2 = nullptr;
  if ((rc = repr_launch<64, 64, 1, 16, 0, true>(a, s)) != LZM_OK) return rc;
  // resblocks2: D1 -> D0 -> D1 (+ D1)
  a.in = D1; a.w = w + L.r2w1; a.winv = w + L.r2s1; a.bias = w + L.r2b1; a.res = nullptr; a.out = D0;
  if ((rc = repr_launch<64, 64, 1, 16, 0, false>(a, s)) != LZM_OK) return rc;
  a.in = D0; a.w = w + L.r2w2; a.winv = w + L.r2s2; a.bias = w + L.r2b2; a.res = D1; a.out = D1;
  if ((rc = repr_launch<64, 64, 1, 16, 0, true>(a, s)) != LZM_OK) return rc;
  // avg pool -> out NCHW [B][64][8][8]
  hipLaunchKernelGGL(repr_avgpool_kernel, dim3(B), dim3(256), 0, s, D1, out, B);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

int lzm_conv_trunk(int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights, const float *actmap,
                   const float *pool, const int32_t *x, const int32_t *action, float *out_latent, float *out_r,
                   float *out_h, void *stream) {
  return lzm_conv_trunk_p(LZM_CONV_F32, B, n_dres, n_pres, r_ch, h_ch, weights, actmap, pool, x, action, out_latent,
                          out_r, out_h, nullptr, stream);
}

}  // extern "C"

extern "C" int lzm_conv_heads(int B, int Kr, int Khd, int off_policy, const float *r, const float *r_scale,
                              const float *r_shift, const float *hd, const float *w1t, const float *b1,
                              const float *w2t, const float *b2, int Vr, int Vv, int A, float *reward, float *value,
                              float *policy, int32_t *norm_words, void *stream) {
  // r == NULL: the prediction heads only (value, policy: initial_inference), reward / norm_words unused
  const bool pred_only = !r;
  if (B <= 0 || (!pred_only && (Kr <= 0 || Kr > kHdRMax || (Kr & 3) || !reward)) || Khd <= 0 || Khd > kHdHMax ||
      off_policy <= 0 || off_policy >= Khd || Khd - off_policy > kHdKMax || off_policy > kHdKMax || Vr <= 0 ||
      Vv <= 0 || A <= 0 || Vr > kHdCols * kHdThreads || Vv > kHdCols * kHdThreads || A > kHdCols * kHdThreads ||
      !hd || !w1t || !b1 || !w2t || !b2 || !value || !policy || (!r_scale) != (!r_shift) || ((uintptr_t)w1t & 15) ||
      (Khd & 3) || (off_policy & 3)) {
    set_err("lzm_conv_heads: bad arguments (Kr <= 1024, head planes <= 2048, K per head <= 1024, supports <= 768, 16-B aligned w1t)");
    return LZM_ERR_ARG;
  }
  HeadsArgs p;
  p.B = B; p.Kr = Kr; p.Khd = Khd;
  p.r = r; p.r_scale = r_scale; p.r_shift = r_shift; p.hd = hd;
  p.src[0] = 0; p.off[0] = 0; p.K[0] = Kr;
  p.src[1] = 1; p.off[1] = 0; p.K[1] = off_policy;
  p.src[2] = 1; p.off[2] = off_policy; p.K[2] = Khd - off_policy;
  p.w1t = w1t; p.b1 = b1; p.w2t = w2t; p.b2 = b2;
  p.Vr = Vr; p.Vv = Vv; p.A = A;
  p.reward = reward; p.value = value; p.policy = policy;
  p.norm_words = pred_only ? nullptr : norm_words; p.norm_nparts = norm_parts(B);
  p.head0 = pred_only ? 1 : 0;
  p.prep_on = 0;
  hipLaunchKernelGGL(conv_heads_kernel, dim3((B + kHdEnvs - 1) / kHdEnvs, pred_only ? 2 : 3), dim3(kHdThreads), 0,
                     (hipStream_t)stream, p);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// The initial inference's prediction heads (lzm_conv_heads with r == NULL) and, in the same launch, the root
// preparation from the policy logits (lzm_roots_prepare's arguments and bits): the policy-head workgroups run
// CRoots::prepare (cnode.cpp:301-358) for their envs from their LDS copy of the logits.
extern "C" int lzm_conv_heads_prepare(lzm_handle *h, int B, int Khd, int off_policy, const float *hd,
                                      const float *w1t, const float *b1, const float *w2t, const float *b2, int Vr,
                                      int Vv, int A, float *value, float *policy, const int32_t *legal,
                                      const int32_t *count, const float *noises, float noise_weight,
                                      const float *rewards, const int32_t *to_play, void *stream) {
  if (!h || h->B != B || h->A != A || A > kHdThreads || !legal || !count || !rewards || !to_play) {
    set_err("lzm_conv_heads_prepare: the handle must have B roots and A <= 256 actions; legal, count, rewards, "
            "to_play required");
    return LZM_ERR_ARG;
  }
  if (B <= 0 || Khd <= 0 || Khd > kHdHMax || off_policy <= 0 || off_policy >= Khd || Khd - off_policy > kHdKMax ||
      off_policy > kHdKMax || Vr <= 0 || Vv <= 0 || Vv > kHdCols * kHdThreads || !hd || !w1t || !b1 || !w2t || !b2 ||
      !value || !policy || ((uintptr_t)w1t & 15) || (Khd & 3) || (off_policy & 3)) {
    set_err("lzm_conv_heads_prepare: bad arguments (head planes <= 2048, K per head <= 1024, supports <= 768, "
            "16-B aligned w1t)");
    return LZM_ERR_ARG;
  }
  HeadsArgs p;
  memset(&p, 0, sizeof(p));
  p.B = B; p.Kr = 0; p.Khd = Khd;
  p.hd = hd;
  p.src[0] = 0; p.off[0] = 0; p.K[0] = 0;
  p.src[1] = 1; p.off[1] = 0; p.K[1] = off_policy;
  p.src[2] = 1; p.off[2] = off_policy; p.K[2] = Khd - off_policy;
  p.w1t = w1t; p.b1 = b1; p.w2t = w2t; p.b2 = b2;
  p.Vr = Vr; p.Vv = Vv; p.A = A;
  p.value = value; p.policy = policy;
  p.norm_nparts = norm_parts(B);
  p.head0 = 1;
  PrepareArgs &q = p.prep;
  q.stat = h->stat; q.meta = h->meta; q.legal = h->legal; q.nlegal = h->nlegal;
  q.legal_in = legal; q.count_in = count; q.to_play = to_play; q.noises = noises; q.rewards = rewards;
  q.logits = policy; q.noise_weight = noise_weight; q.B = h->B; q.A = h->A;
  p.prep_on = 1;
  hipLaunchKernelGGL(conv_heads_kernel, dim3((B + kHdEnvs - 1) / kHdEnvs, 2), dim3(kHdThreads), 0, (hipStream_t)stream,
                     p);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// Whole-search launch for the conv MuZero networks (lzm_search_conv.h): one workgroup per root,
// every simulation inside the kernel. The grid must be co-resident (one workgroup per CU, B <= CUs):
// parity-mode roots wait on their predecessors' depth flags.
extern "C" int lzm_search_conv(lzm_handle *h, int num_simulations, int pb_c_base, float pb_c_init, float discount,
                               float *minmax, const uint32_t *seeds, const int32_t *vtp_in, float *latent_pool,
                               const float *trunk_w, const float *actmap, int n_dres, int n_pres, int r_ch, int h_ch,
                               const float *w1t, const float *b1, const float *w2q, const float *b2, int Kr, int Khd,
                               int off_policy, int Vr, int Vv, int categorical, int32_t *rec_x, int32_t *rec_a,
                               int32_t *rec_len, float *rec_decoded, float *rec_logits, void *stream) {
  const int S = num_simulations;
  if (!h || !minmax || (!seeds && !h->step_count) || !vtp_in || !latent_pool || !trunk_w || !actmap || !w1t || !b1 ||
      !w2q || !b2 ||
      S <= 0) {
    set_err("lzm_search_conv: null argument or no simulations");
    return LZM_ERR_ARG;
  }
  if (h->flags & LZM_TREE_EZ) {
    set_err("lzm_search_conv: MuZero trees only");
    return LZM_ERR_ARG;
  }
  if (n_dres < 0 || n_pres < 0 || r_ch <= 0 || r_ch > 32 || h_ch <= 0 || h_ch > 32 || Kr != r_ch * 64 ||
      Khd != h_ch * 64 || off_policy <= 0 || off_policy >= Khd || off_policy > kHdKMax || Khd - off_policy > kHdKMax ||
      (off_policy % 128) || (Kr % 128) || (Khd % 128) || Vr <= 0 || Vv <= 0 || Vr > 1024 || Vv > 1024 ||
      (!categorical && (Vr != 1 || Vv != 1)) ||
      (((uintptr_t)trunk_w | (uintptr_t)actmap | (uintptr_t)w1t | (uintptr_t)w2q | (uintptr_t)latent_pool) & 15)) {
    set_err("lzm_search_conv: unsupported network shape (64x8x8 latent, <= 32 reward / head planes, K per head a "
            "multiple of 128 and <= 1024, supports <= 1024, 16-B aligned weights and pool)");
    return LZM_ERR_ARG;
  }
  if (S > h->sims_cap) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv: %d simulations > reserved %d (lzm_reserve)", S, h->sims_cap);
    return LZM_ERR_CAPACITY;
  }
  // one workgroup per root; roots beyond the CUs queue behind the first ones (their look-back waits only on
  // lower roots: lzm_search_conv.h sc_lookback)
  if (h->B > kScMaxRoots) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv: %d roots > %d", h->B, kScMaxRoots);
    return LZM_ERR_ARG;
  }
  int rc = fill_lut(h, pb_c_base, pb_c_init);
  if (rc != LZM_OK) return rc;
  const bool fast = (h->flags & LZM_RNG_FAST) != 0;
  if (!fast) {
    rc = ensure_coef(h, h->B * (S + 1) + 64);
    if (rc != LZM_OK) return rc;
  }
  rc = ensure_flags(h, S, h->B);
  if (rc != LZM_OK) return rc;
  ConvSearchArgs p;
  memset(&p, 0, sizeof(p));
  p.stat = h->stat; p.meta = h->meta; p.legal = h->legal; p.nlegal = h->nlegal;
  p.path = h->path; p.path_act = h->path_act; p.pathlen = h->pathlen; p.lut = h->lut;
  p.B = h->B; p.A = h->A; p.cap = h->cap; p.lut_n = h->lut_n; p.depth_cap = h->depth_cap;
  p.S = S; p.disc = discount; p.seeds = seeds; p.vtp_in = vtp_in; p.minmax = (float4 *)minmax; p.pool = latent_pool;
  p.w = trunk_w; p.actmap = actmap; p.n_dres = n_dres; p.n_pres = n_pres; p.r_ch = r_ch; p.h_ch = h_ch;
  p.w1t = w1t; p.b1 = b1; p.w2q = w2q; p.b2 = b2; p.Kr = Kr; p.Khd = Khd; p.off_policy = off_policy;
  p.Vr = Vr; p.Vv = Vv; p.categorical = categorical ? 1 : 0;
  p.coef = h->coef; p.coef_positions = h->coef_positions; p.pow16807 = h->pow16807;
  p.flags = h->lb_flags; p.epoch = h->epoch; p.err = h->err; p.sdiag = h->search_diag; p.fast = fast ? 1 : 0;
  p.rec_x = rec_x; p.rec_a = rec_a; p.rec_len = rec_len; p.rec_dec = rec_decoded; p.rec_logits = rec_logits;
  p.step_count = h->step_count; p.step_base = h->step_base; p.step_inc = h->step_inc; p.step_fresh = h->step_fresh;
  p.step_delta = h->step_delta; p.out_dist = h->step_dist; p.out_values = h->step_vals;
  // dynamic LDS plan (float offsets, 16-B aligned): the two split-fp16 activation buffers first
  size_t o = (size_t)2 * kBxBuf / 2;
  p.off_stat = (int)o; o += (size_t)h->cap * 4;
  p.off_meta = (int)o; o += (size_t)h->cap * 4;
  p.off_val = (int)o; o += round4((size_t)h->cap);
  p.off_lut = (int)o; o += round4((size_t)2 * h->lut_n);
  p.off_legal = (int)o; o += round4((size_t)h->A + 1);
  p.off_path = (int)o; o += round4((size_t)h->depth_cap);
  p.off_pact = (int)o; o += round4((size_t)h->depth_cap);
  p.pbt_rows = 0;  // (no pb_c table: the MuZero conv walk divides, same bits)
  p.off_pbt = (int)o;
  p.off_r = (int)o; o += round4((size_t)Kr);
  p.off_hd = (int)o; o += round4((size_t)Khd);
  p.off_hid = (int)o; o += 96;
  p.off_part = (int)o; o += 3 * kHdParts * 32;
  p.off_lg = (int)o; o += round4((size_t)Vr + Vv + h->A);
  p.off_seed = (int)o; o += round4((size_t)S + 32);
  p.off_lmax = (int)o; o += round4((size_t)S + 1);
  if (o * sizeof(float) > kMaxLds) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv: %zu B of LDS needed (tree too large: lower num_simulations)",
             o * sizeof(float));
    return LZM_ERR_ARG;
  }
  // the head hidden layers' first half-head resident in LDS when it fits and every root has a CU of its own
  // (more roots than CUs: the smaller footprint lets two workgroups share one)
  constexpr size_t kPinFloats = (size_t)kHdParts * 16 * 32 * 4;
  const char *pin_env = getenv("LZM_CONV_PIN");
  const int pin_max = pin_env ? atoi(pin_env) : 1;
  p.off_wpin = (int)o;
  p.npin = 0;
  while (p.npin < pin_max && p.npin < 6 && h->B <= device_cus() && (o + kPinFloats) * sizeof(float) <= kMaxLds) {
    o += kPinFloats;
    ++p.npin;
  }
  const size_t lds = o * sizeof(float);
  const bool stamps = getenv("LZM_PHASE_TIMING") && atoi(getenv("LZM_PHASE_TIMING")) > 0;
  if (stamps && !h->phase) {
    LZM_HIP(hipMalloc(&h->phase, (64 + 1024) * sizeof(unsigned long long)));
    LZM_HIP(hipMemset(h->phase, 0, (64 + 1024) * sizeof(unsigned long long)));
  }
  p.stamps = stamps ? h->phase : nullptr;
  auto fn = stamps ? (fast ? search_conv_kernel<kBxAhead, true, true> : search_conv_kernel<kBxAhead, false, true>)
                   : (fast ? search_conv_kernel<kBxAhead, true> : search_conv_kernel<kBxAhead, false>);
  hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fn, dim3(h->B), dim3(kScThreads), lds, (hipStream_t)stream, p);
    e = hipGetLastError();
  }
  LZM_HIP(e);
  return LZM_OK;
}

// Whole-search launch for the conv EfficientZero networks (lzm_search_conv.h, EZ instantiation): the
// MuZero launch's flow plus the reward LSTM as split-K tiles spread over the grid (G = max(B, 2 T)
// workgroups, one per CU, co-resident: the tiles wait on the roots' LSTM input rows and the roots on
// their rows' tiles inside the launch).
extern "C" int lzm_search_conv_ez(lzm_handle *h, int num_simulations, int pb_c_base, float pb_c_init, float discount,
                                  float *minmax, const uint32_t *seeds, const int32_t *vtp_in, float *latent_pool,
                                  float *hpool, float *cpool, int H, int horizon, const float *trunk_w,
                                  const float *actmap, int n_dres, int n_pres, int r_ch, int h_ch,
                                  const float *lstm_frag, const float *lstm_bias, const float *vp_s, const float *vp_t,
                                  const float *w1t, const float *b1, const float *w2q, const float *b2, int Khd,
                                  int off_policy, int Vr, int Vv, int categorical, int32_t *rec_x, int32_t *rec_a,
                                  int32_t *rec_len, float *rec_decoded, float *rec_logits, int32_t *rec_reset,
                                  void *stream) {
  const int S = num_simulations;
  if (!h || !minmax || (!seeds && !h->step_count) || !vtp_in || !latent_pool || !hpool || !cpool || !trunk_w ||
      !actmap || !lstm_frag ||
      !lstm_bias || !vp_s || !vp_t || !w1t || !b1 || !w2q || !b2 || S <= 0) {
    set_err("lzm_search_conv_ez: null argument or no simulations");
    return LZM_ERR_ARG;
  }
  if (!(h->flags & LZM_TREE_EZ)) {
    set_err("lzm_search_conv_ez: EfficientZero trees only");
    return LZM_ERR_ARG;
  }
  const int Kx = r_ch * 64 + H;
  if (n_dres < 0 || n_pres < 0 || r_ch <= 0 || r_ch > 32 || h_ch <= 0 || h_ch > 32 || Khd != h_ch * 64 ||
      off_policy <= 0 || off_policy >= Khd || off_policy > kHdKMax || Khd - off_policy > kHdKMax || (off_policy % 128) ||
      (Khd % 128) || H <= 0 || H % kLsUnits || H % 128 || H > kHdKMax || H / kLsUnits > 64 || Kx % (2 * kLsKc) ||
      horizon <= 0 || Vr <= 0 || Vv <= 0 || Vr > 1024 || Vv > 1024 || (!categorical && (Vr != 1 || Vv != 1)) ||
      S > 4094 ||
      (((uintptr_t)trunk_w | (uintptr_t)actmap | (uintptr_t)w1t | (uintptr_t)w2q | (uintptr_t)latent_pool |
        (uintptr_t)hpool | (uintptr_t)cpool | (uintptr_t)lstm_frag | (uintptr_t)vp_s | (uintptr_t)vp_t) & 15)) {
    set_err("lzm_search_conv_ez: unsupported network shape (64x8x8 latent, <= 32 reward / head planes, K per head a "
            "multiple of 128 and <= 1024, LSTM width a multiple of 128, (r_ch * 64 + H) % 128 == 0, horizon > 0, "
            "16-B aligned weights and pools) or more than 4094 simulations");
    return LZM_ERR_ARG;
  }
  if (S > h->sims_cap) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv_ez: %d simulations > reserved %d (lzm_reserve)", S, h->sims_cap);
    return LZM_ERR_CAPACITY;
  }
  // LZM_RESIDENCY_CUS=<n> caps the CU count this check assumes (tests: force the refusal)
  int cus = device_cus();
  if (const char *ov = getenv("LZM_RESIDENCY_CUS"))
    if (atoi(ov) > 0) cus = std::min(cus, atoi(ov));
  const int B = h->B, nmb = (B + kLsRows - 1) / kLsRows, T = nmb * (H / kLsUnits), G = std::max(B, 2 * T);
  if (B > 256 || G > cus) {
    snprintf(g_err, sizeof(g_err),
             "lzm_search_conv_ez: %d workgroups (%d roots, %d LSTM tiles x 2) > min(%d CUs) or B > 256 (the grid is "
             "co-resident)", G, B, T, cus);
    return LZM_ERR_RESIDENCY;
  }
  int rc = fill_lut(h, pb_c_base, pb_c_init);
  if (rc != LZM_OK) return rc;
  const bool fast = (h->flags & LZM_RNG_FAST) != 0;
  if (!fast) {
    rc = ensure_coef(h, B * (S + 1) + 64);
    if (rc != LZM_OK) return rc;
  }
  rc = ensure_flags(h, S, B);
  if (rc != LZM_OK) return rc;
  // hand-off workspace, grown on demand (flags zeroed: epoch 0 never matches)
  const size_t f_xin = round4((size_t)B * Kx), f_h1 = round4((size_t)B * H), f_part = (size_t)T * kLpThreads * 16;
  const size_t flag_words = (size_t)S * B + 2 * (size_t)S * T;
  const size_t need = (f_xin + f_h1 + f_part) * sizeof(float) + flag_words * sizeof(unsigned long long);
  if (h->ez_ws_bytes < need) {
    dfree(h->ez_ws);
    h->ez_ws = nullptr;
    h->ez_ws_bytes = 0;
    LZM_HIP(hipMalloc(&h->ez_ws, need));
    LZM_HIP(hipMemset(h->ez_ws, 0, need));
    h->ez_ws_bytes = need;
  }
  float *wsf = reinterpret_cast<float *>(h->ez_ws);
  unsigned long long *wsl = reinterpret_cast<unsigned long long *>(wsf + f_xin + f_h1 + f_part);
  ConvSearchArgs p;
  memset(&p, 0, sizeof(p));
  p.stat = h->stat; p.meta = h->meta; p.legal = h->legal; p.nlegal = h->nlegal;
  p.path = h->path; p.path_act = h->path_act; p.pathlen = h->pathlen; p.lut = h->lut;
  p.B = B; p.A = h->A; p.cap = h->cap; p.lut_n = h->lut_n; p.depth_cap = h->depth_cap;
  p.S = S; p.disc = discount; p.seeds = seeds; p.vtp_in = vtp_in; p.minmax = (float4 *)minmax; p.pool = latent_pool;
  p.w = trunk_w; p.actmap = actmap; p.n_dres = n_dres; p.n_pres = n_pres; p.r_ch = r_ch; p.h_ch = h_ch;
  p.w1t = w1t; p.b1 = b1; p.w2q = w2q; p.b2 = b2; p.Kr = H; p.Khd = Khd; p.off_policy = off_policy;
  p.Vr = Vr; p.Vv = Vv; p.categorical = categorical ? 1 : 0;
  p.coef = h->coef; p.coef_positions = h->coef_positions; p.pow16807 = h->pow16807;
  p.flags = h->lb_flags; p.epoch = h->epoch; p.err = h->err; p.sdiag = h->search_diag; p.fast = fast ? 1 : 0;
  p.rec_x = rec_x; p.rec_a = rec_a; p.rec_len = rec_len; p.rec_dec = rec_decoded; p.rec_logits = rec_logits;
  p.step_count = h->step_count; p.step_base = h->step_base; p.step_inc = h->step_inc; p.step_fresh = h->step_fresh;
  p.step_delta = h->step_delta; p.out_dist = h->step_dist; p.out_values = h->step_vals;
  p.rec_reset = rec_reset;
  p.xin = wsf; p.h1g = wsf + f_xin; p.kpart = wsf + f_xin + f_h1;
  p.xflags = wsl; p.tflags = wsl + (size_t)S * B; p.pflags = wsl + (size_t)S * B + (size_t)S * T;
  p.Kx = Kx; p.H = H; p.horizon = horizon; p.hpool = hpool; p.cpool = cpool;
  p.lwfrag = reinterpret_cast<const uint16_t *>(lstm_frag); p.lwinv = lstm_frag + ls_frag_floats(Kx, H);
  p.lbias = lstm_bias; p.vp_s = vp_s; p.vp_t = vp_t;
  p.nmb = nmb; p.T = T;
  // dynamic LDS plan (float offsets, 16-B aligned): the activation buffers / LSTM stage buffers first
  size_t o = std::max((size_t)2 * kBxBuf / 2, (size_t)kLsLdsBytes / 4);
  p.off_stat = (int)o; o += (size_t)h->cap * 4;
  p.off_meta = (int)o; o += (size_t)h->cap * 4;
  p.off_val = (int)o; o += round4((size_t)h->cap);
  p.off_lut = (int)o; o += round4((size_t)2 * h->lut_n);
  p.off_legal = (int)o; o += round4((size_t)h->A + 1);
  p.off_path = (int)o; o += round4((size_t)h->depth_cap);
  p.off_pact = (int)o; o += round4((size_t)h->depth_cap);
  p.pbt_rows = ((size_t)h->lut_n * (h->lut_n + 1) / 2 <= 4096) ? h->lut_n : 0;
  p.off_pbt = (int)o; o += round4((size_t)p.pbt_rows * (p.pbt_rows + 1) / 2);
  p.off_r = (int)o; o += round4((size_t)H);
  p.off_hd = (int)o; o += round4((size_t)Khd);
  p.off_hid = (int)o; o += 96;
  p.off_part = (int)o; o += 3 * kHdParts * 32;
  p.off_lg = (int)o; o += round4((size_t)Vr + Vv + h->A);
  p.off_seed = (int)o; o += round4((size_t)S + 32);
  p.off_lmax = (int)o; o += round4((size_t)S + 1);
  const size_t lds = o * sizeof(float);
  if (lds > kMaxLds) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv_ez: %zu B of LDS needed (tree too large: lower num_simulations)",
             lds);
    return LZM_ERR_ARG;
  }
  const bool stamps = getenv("LZM_PHASE_TIMING") && atoi(getenv("LZM_PHASE_TIMING")) > 0;
  if (stamps && !h->phase) {
    LZM_HIP(hipMalloc(&h->phase, (64 + 1024) * sizeof(unsigned long long)));
    LZM_HIP(hipMemset(h->phase, 0, (64 + 1024) * sizeof(unsigned long long)));
  }
  p.stamps = stamps ? h->phase : nullptr;
  auto fn = stamps ? (fast ? search_conv_ez_kernel<kBxAheadEz, true, true> : search_conv_ez_kernel<kBxAheadEz, false, true>)
                   : (fast ? search_conv_ez_kernel<kBxAheadEz, true> : search_conv_ez_kernel<kBxAheadEz, false>);
  LZM_HIP(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // The roots wait on LSTM tiles and the tiles on roots inside the launch, so every workgroup must be
  // resident at once. The check is static: resident workgroups per CU at this LDS / register use (the
  // occupancy API) x the CUs must cover the grid, else LZM_ERR_RESIDENCY and nothing ran (the caller takes
  // the generic per-simulation path). It cannot see other work on the GPU (a learner on another stream, a
  // second rank on the same GPU): every hand-off wait in the kernel is bounded and a timeout is counted in
  // the tree's error word (lzm_check_errors raises), never a hang. The launch is a plain one, eager and
  // captured alike: the cooperative launch it replaced applies the same static occupancy check (it is
  // not a residency guarantee against other streams), cannot be captured into a HIP graph, and its
  // runtime state was the one difference from the MuZero conv search in the EZ trace that faulted in
  // exit() after rocprofv3 finalised (profiles/r05/README.md).
  int per_cu = 0;
  LZM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)fn, kScThreads, lds));
  if ((long long)per_cu * cus < G) {
    snprintf(g_err, sizeof(g_err), "lzm_search_conv_ez: %d workgroups > %d resident (%d per CU x %d CUs)", G,
             per_cu * cus, per_cu, cus);
    return LZM_ERR_RESIDENCY;
  }
  hipLaunchKernelGGL(fn, dim3(G), dim3(kScThreads), lds, (hipStream_t)stream, p);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

// Test support: n workgroups that each occupy a CU (the whole LDS) for `usec` microseconds of the 100 MHz real-time
// clock, then exit — another stream's kernel holding CUs while a co-resident grid launches (tests only).
__global__ void hold_cu_kernel(unsigned long long ticks) {
  extern __shared__ uint4 hold_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) hold_lds[0] = uint4{0u, 0u, 0u, 0u};
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

extern "C" int lzm_debug_hold_cus(int n, int usec, void *stream) {
  if (n <= 0 || n > 4096 || usec <= 0 || usec > 2000000) {
    set_err("lzm_debug_hold_cus: 1..4096 workgroups for up to 2 s");
    return LZM_ERR_ARG;
  }
  static hipError_t attr = hipFuncSetAttribute((const void *)hold_cu_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)kMaxLds);
  LZM_HIP(attr);
  hipLaunchKernelGGL(hold_cu_kernel, dim3(n), dim3(64), kMaxLds, (hipStream_t)stream, (unsigned long long)usec * 100ull);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_ez_lstm_input(int B, int Kr, int H, const float *r, const float *hpool, const int32_t *x, float *xin,
                                 void *stream) {
  if (B <= 0 || Kr <= 0 || H <= 0 || (Kr & 3) || (H & 3) || !r || !hpool || !x || !xin ||
      (((uintptr_t)r | (uintptr_t)hpool | (uintptr_t)xin) & 15)) {
    set_err("lzm_ez_lstm_input: bad arguments (Kr, H multiples of 4, 16-B aligned buffers)");
    return LZM_ERR_ARG;
  }
  const long long n = (long long)B * ((Kr + H) >> 2);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(ez_lstm_input_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, Kr, H, r, hpool, x, xin);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_ez_lstm_cell(int B, int H, const float *gates, const float *cpool, const int32_t *x,
                                const int32_t *search_len, int horizon, float *h1, float *c1, float *hslot,
                                float *cslot, void *stream) {
  if (B <= 0 || H <= 0 || (H & 3) || !gates || !cpool || !x || !search_len || !h1 || !c1 || !hslot || !cslot ||
      (((uintptr_t)gates | (uintptr_t)cpool | (uintptr_t)h1 | (uintptr_t)c1 | (uintptr_t)hslot | (uintptr_t)cslot) & 15)) {
    set_err("lzm_ez_lstm_cell: bad arguments (H multiple of 4, 16-B aligned buffers)");
    return LZM_ERR_ARG;
  }
  const long long n = (long long)B * (H >> 2);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(ez_lstm_cell_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, H, gates, cpool, x,
                     search_len, horizon, h1, c1, hslot, cslot);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int64_t lzm_ez_lstm_frag_floats(int K, int H) {
  if (K <= 0 || H <= 0 || K % kLsKc || H % kLsUnits) return -1;
  return ls_frag_floats(K, H) + 4 * (int64_t)H;  // the fragments, then the 4H column scales
}

extern "C" int lzm_ez_lstm_prepare(int K, int H, const float *W, float *out) {
  if (lzm_ez_lstm_frag_floats(K, H) < 0 || !W || !out) {
    set_err("lzm_ez_lstm_prepare: need K % 64 == 0, H % 16 == 0 and buffers");
    return LZM_ERR_ARG;
  }
  ls_pack(W, K, H, out);
  return LZM_OK;
}

static unsigned long long *g_ls_stamps = nullptr;  // diagnostics: lzm_debug_lstm_stamps
extern "C" int lzm_debug_lstm_stamps(void *buf) {
  g_ls_stamps = reinterpret_cast<unsigned long long *>(buf);
  return LZM_OK;
}

extern "C" int64_t lzm_ez_lstm_workspace_bytes(int B, int H) {
  if (B <= 0 || H <= 0 || H % kLsUnits) return -1;
  const int64_t tiles = (int64_t)((B + kLsRows - 1) / kLsRows) * (H / kLsUnits);
  return tiles * kLsPartFloats * 4 + tiles * 4;
}

extern "C" int lzm_ez_lstm_step(int B, int K, int H, const float *xin, const int32_t *xscale, const float *wfrag,
                                const float *bias, const float *cpool, const int32_t *x, const int32_t *search_len,
                                int horizon, float *h1, float *c1, float *hslot, float *cslot, void *workspace,
                                int32_t *err, int32_t *range_err, void *stream) {
  if (B <= 0 || lzm_ez_lstm_frag_floats(K, H) < 0 || !xin || !xscale || !wfrag || !bias || !cpool || !x || !search_len || !h1 ||
      !c1 || !hslot || !cslot || (((uintptr_t)xin | (uintptr_t)wfrag | (uintptr_t)workspace) & 15) ||
      (workspace && !err)) {
    set_err("lzm_ez_lstm_step: bad arguments (K % 64 == 0, H % 16 == 0, 16-B aligned xin / fragments / workspace, "
            "an error word with the workspace)");
    return LZM_ERR_ARG;
  }
  LstmArgs a;
  a.B = B; a.K = K; a.H = H; a.nmb = (B + kLsRows - 1) / kLsRows;
  a.xin = xin; a.xscale = xscale; a.range_err = range_err;
  a.wf = reinterpret_cast<const uint4 *>(wfrag); a.winv = wfrag + ls_frag_floats(K, H);
  a.bias = bias; a.cpool = cpool; a.x = x;
  a.search_len = search_len; a.horizon = horizon; a.h1 = h1; a.c1 = c1; a.hslot = hslot; a.cslot = cslot;
  const int tiles = a.nmb * (H / kLsUnits);
  // split K in two when a workspace is given and every workgroup is resident at once (the lower K
  // half waits for the upper; one 512-thread workgroup per CU by its LDS)
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 0;
  a.splitk = (workspace && K % (2 * kLsKc) == 0 && 2 * tiles <= cus) ? 2 : 1;
  a.part = reinterpret_cast<float *>(workspace);
  a.flags = workspace ? reinterpret_cast<uint32_t *>(a.part + (size_t)tiles * kLsPartFloats) : nullptr;
  a.err = err;
  a.stamps = g_ls_stamps;
  static bool attr = false;
  if (!attr) {
    LZM_HIP(hipFuncSetAttribute((const void *)ez_lstm_gemm_cell_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kLsLdsBytes));
    attr = true;
  }
  hipLaunchKernelGGL(ez_lstm_gemm_cell_kernel, dim3(tiles * a.splitk), dim3(kLsThreads), kLsLdsBytes,
                     (hipStream_t)stream, a);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_mlp_initial_inference(int B, int O, int H, int F, int V, int A, int group, const float *obs,
                                         const float *weights, const int64_t *offsets, float *latent, float *value,
                                         float *policy, void *stream) {
  if (B <= 0 || O <= 0 || O > kIiMaxW || H <= 0 || H > kIiMaxW || F <= 0 || F > 256 || V <= 0 || V > kIiMaxW ||
      A <= 0 || A > kIiMaxW || group <= 0 || H % group || !obs || !weights || !offsets || !latent || !value ||
      !policy) {
    set_err("lzm_mlp_initial_inference: bad arguments (widths <= 1024, head hidden <= 256, H % group == 0)");
    return LZM_ERR_ARG;
  }
  IiArgs p;
  p.B = B; p.O = O; p.H = H; p.F = F; p.V = V; p.A = A; p.group = group;
  p.obs = obs;
  for (int l = 0; l < kIiLayers; ++l) {
    p.w[l] = l < 8 ? weights + offsets[2 * l] : nullptr;
    p.b[l] = l < 8 ? weights + offsets[2 * l + 1] : nullptr;
  }
  p.latent = latent; p.value = value; p.policy = policy;
  hipLaunchKernelGGL(initial_inference_kernel<false>, dim3((B + kIiEnvs - 1) / kIiEnvs), dim3(kIiThreads), 0,
                     (hipStream_t)stream, p, PrepareArgs{});
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_mlp_initial_inference_prepare(lzm_handle *h, int B, int O, int H, int F, int V, int A, int group,
                                                 const float *obs, const float *weights, const int64_t *offsets,
                                                 float *latent, float *value, float *policy, const int32_t *legal,
                                                 const int32_t *count, const float *noises, float noise_weight,
                                                 const float *rewards, const int32_t *to_play, void *stream) {
  if (!h || h->B != B || h->A != A || !legal || !count || !rewards || !to_play) {
    set_err("lzm_mlp_initial_inference_prepare: the handle must have B roots and A actions; legal, count, rewards, "
            "to_play required");
    return LZM_ERR_ARG;
  }
  if (B <= 0 || O <= 0 || O > kIiMaxW || H <= 0 || H > kIiMaxW || F <= 0 || F > 256 || V <= 0 || V > kIiMaxW ||
      A <= 0 || A > kIiMaxW || group <= 0 || H % group || !obs || !weights || !offsets || !latent || !value ||
      !policy) {
    set_err("lzm_mlp_initial_inference_prepare: bad arguments (widths <= 1024, head hidden <= 256, H % group == 0)");
    return LZM_ERR_ARG;
  }
  IiArgs p;
  p.B = B; p.O = O; p.H = H; p.F = F; p.V = V; p.A = A; p.group = group;
  p.obs = obs;
  for (int l = 0; l < kIiLayers; ++l) {
    p.w[l] = l < 8 ? weights + offsets[2 * l] : nullptr;
    p.b[l] = l < 8 ? weights + offsets[2 * l + 1] : nullptr;
  }
  p.latent = latent; p.value = value; p.policy = policy;
  PrepareArgs q;
  q.stat = h->stat; q.meta = h->meta; q.legal = h->legal; q.nlegal = h->nlegal;
  q.legal_in = legal; q.count_in = count; q.to_play = to_play; q.noises = noises; q.rewards = rewards;
  q.logits = policy; q.noise_weight = noise_weight; q.B = h->B; q.A = h->A;
  hipLaunchKernelGGL(initial_inference_kernel<true>, dim3((B + kIiEnvs - 1) / kIiEnvs), dim3(kIiThreads), 0,
                     (hipStream_t)stream, p, q);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_set_reuse(lzm_handle *h, const int32_t *true_action, const float *reuse_value) {
  if (!h || (!true_action) != (!reuse_value)) {
    set_err("lzm_set_reuse: both arrays or neither");
    return LZM_ERR_ARG;
  }
  h->reuse_action = true_action;
  h->reuse_value = reuse_value;
  return LZM_OK;
}

extern "C" int lzm_set_norm_words(lzm_handle *h, const int32_t *words) {
  if (!h) return LZM_ERR_ARG;
  h->ext_norm = words;
  return LZM_OK;
}

// Traverse seeds of one collect step (SURVEY.md §8(d) rule, lightzero_amd.collect.DeviceSearchStep):
// seeds[k] = (base + count * S + k) mod 10^6, count read on the device (a captured graph replays it).
__global__ void seed_sequence_kernel(const int64_t *count, long long base, int S, int32_t *seeds) {
  const long long c = *count;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < S; k += gridDim.x * blockDim.x)
    seeds[k] = (int32_t)((base + c * (long long)S + k) % 1000000ll);
}

extern "C" int lzm_seed_sequence(const int64_t *count, int64_t base, int S, int32_t *seeds, void *stream) {
  if (!count || !seeds || S <= 0 || base < 0) {
    set_err("lzm_seed_sequence: bad arguments");
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(seed_sequence_kernel, dim3((S + 255) / 256), dim3(256), 0, (hipStream_t)stream, count,
                     (long long)base, S, seeds);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}

extern "C" int lzm_get_root_outputs(lzm_handle *h, int32_t *dist, float *values, void *stream) {
  if (!h || !dist || !values) {
    set_err("lzm_get_root_outputs: null argument");
    return LZM_ERR_ARG;
  }
  hipLaunchKernelGGL(root_outputs_kernel, dim3((h->B + 255) / 256), dim3(256), 0, (hipStream_t)stream, view(h), dist,
                     values);
  LZM_CHECK_LAUNCH();
  return LZM_OK;
}
