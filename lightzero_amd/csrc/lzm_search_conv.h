// lzm_search_conv.h — one launch = one whole MuZero search for the conv Atari networks
// (BASELINE.json config 5: Breakout MuZero, 64 x 8 x 8 latent, support 601; one GPU's 256-env shard).
//
// Replaces the generic path's four launches per simulation (look-back traverse, conv trunk, head
// MLPs, decode + backup; mcts_ctree.py:255-321 around muzero_model.py:241-373's recurrent step)
// with ONE launch for all S simulations: workgroup b owns root b for the whole search. Its tree
// slice (node records, value cache, pUCT table, path) lives in LDS; per simulation
//   1. wave 0 walks the tree (descend_wave, bit-exact with cbatch_traverse). Parity mode: the
//      reference's single rand() stream gives root b the draws at positions sum_{q<b} depth_q, so
//      the walk first runs draw-free, publishes the depth in a {epoch, depth} flag and, only when a
//      draw value is needed, looks back over its predecessors' flags (lzm_traverse_lb.h's scheme,
//      inside the persistent kernel);
//   2. the four waves run the split-fp16 MFMA trunk (lzm_conv.h: dynamics conv + action map,
//      residual blocks, reward 1x1, prediction blocks, value/policy 1x1) from the leaf's parent
//      latent pool[x][b] (HBM: every expanded node's latent is 16 KB, written by this workgroup in an
//      earlier simulation, so it is an L2 hit on this XCD) and file the next latent in pool[k+1][b];
//      the reward / head planes stay in LDS;
//   3. the reward / value / policy head MLPs (lzm_heads.h's arithmetic, weights from L2);
//   4. waves 0 / 1 decode the reward / value supports (InverseScalarTransform: softmax, expectation,
//      h^-1), wave 0 expands the leaf and backs the value up (expand_wave, backup_wave).
// Every arithmetic step is the generic path's own device code in the same order, so the fused
// search equals the generic one bit for bit (tests/test_gpu_conv.py).
//
// ensure_softmax (scaling_transform.py:36-62) is a batch-wide verdict per simulation: softmax is
// skipped only when EVERY row sums to 1. A workgroup whose own row fails the check knows the
// verdict (softmax); one whose own row passes cannot decide alone and counts an integrity error
// (sdiag[0], raised by lzm_check_errors) instead of waiting on the whole grid — a network whose
// raw support logits sum to 1 within 1e-5 does not occur in practice.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_conv.h"
#include "lzm_heads.h"
#include "lzm_lstm.h"
#include "lzm_search_mlp.h"
#include "lzm_tree.h"

namespace lzm {

constexpr int kScThreads = 256;
constexpr int kScMaxRoots = 1024;  // search_conv_kernel: roots per launch (one workgroup each, queued past the CUs)

struct ConvSearchArgs {
  // tree (HBM, whole batch; the kernel stages root b's slice)
  NodeStat *stat;
  NodeMeta *meta;
  const int32_t *legal, *nlegal;
  int32_t *path, *path_act, *pathlen;
  const float2 *lut;
  int B, A, cap, lut_n, depth_cap, pbt_rows;
  // search
  int S;
  float disc;
  const uint32_t *seeds;  // [S]
  const int32_t *vtp_in;  // [B]
  float4 *minmax;         // [B]
  float *pool;            // [S+1][B][4096]
  // trunk (split-fp16 layout, lzm_conv_trunk_prepare_p) and heads (lzm_heads.h layouts)
  const float *w, *actmap;
  int n_dres, n_pres, r_ch, h_ch;
  const float *w1t, *b1, *w2q, *b2;  // w2q: the output layer as [8][N2][4] (k4-major float4s, 16-B aligned)
  int Kr, Khd, off_policy, Vr, Vv, categorical;
  // parity-mode draws
  const uint32_t *coef;
  int coef_positions;
  const uint32_t *pow16807;
  unsigned long long *flags;  // [S][B] {epoch, depth}
  uint32_t *epoch;            // [2]
  int32_t *err;               // sticky: [0] look-back spin timeouts, [1] draw-table overflows
  int32_t *sdiag;             // [0] undecidable ensure_softmax verdicts (integrity errors)
  int fast;
  // optional per-simulation record
  int32_t *rec_x, *rec_a, *rec_len;
  float *rec_dec, *rec_logits;
  int32_t *rec_reset;  // EfficientZero: is_reset [S][B]
  // EfficientZero (search_conv_ez_kernel): the reward LSTM of the recurrent step (lzm_lstm.h)
  float *xin;             // [B][Kx] LSTM input rows [reward planes | leaf hidden state] (sc1 hand-off)
  int Kx, H, horizon;     // Kx = r_ch * 64 + H; lstm_horizon_len
  float *hpool, *cpool;   // [S + 1][B][H] state pools (slot 0 = the roots' state)
  const uint16_t *lwfrag; // gate weights, split-fp16 fragments (lzm_ez_lstm_prepare)
  const float *lwinv;     // [4H] their column scales 2^-e_j (after the fragments)
  const float *lbias;     // [4H] b_ih + b_hh
  const float *vp_s, *vp_t;  // value-prefix BatchNorm as an affine map (relu(h1 * s + t) feeds the head)
  float *h1g;             // [B][H] unmasked LSTM outputs (sc1 hand-off, tile -> root)
  float *kpart;           // [T][kLpThreads * 16] split-K partial sums (sc1 hand-off, upper -> lower half)
  unsigned long long *xflags, *tflags, *pflags;  // [S][B], [S][T], [S][T] {epoch, payload} words
  int nmb, T;             // row blocks of 64, tiles (nmb * H / 16)
  unsigned long long *stamps;  // STAMPS instantiation only
  // collect-step mode (lzm_search_set_step on the handle; lightzero_amd.collect): the seeds of this step from
  // the device step counter ((base + count * S + k) mod 10^6, seed_sequence_kernel's rule), fresh min-max
  // bounds, the root outputs (visit counts per legal action, the root value) and the counter advanced by the
  // last workgroup — the launches around the search folded into it
  int64_t *step_count;
  long long step_base;
  int step_inc, step_fresh;
  float step_delta;
  int32_t *out_dist;
  float *out_values;
  // dynamic LDS plan: float offsets (the two activation buffers come first)
  int off_stat, off_meta, off_val, off_lut, off_legal, off_path, off_pact, off_pbt, off_r, off_hd, off_hid, off_part,
      off_lg, off_seed, off_lmax;
  int off_wpin, npin;  // LDS copy of the first npin half-heads of w1t (sc_heads_hidden_rs), 64 KiB each
};

// Bounded waits of the one-launch conv searches (their grid must be co-resident; the host checks the static
// occupancy bound, which cannot see another stream's kernel holding CUs): a wait gives up after kScSpinTicks
// of the 100 MHz real-time clock (200 ms: a whole 256 x 50 search takes ~3 ms), counts err[0] and raises the
// launch's abort word err[5], after which every other wait of the launch returns at once — a grid that is not
// resident ends after ~one timeout with a search the host discards (mcts_ctree: the eager search restores
// the tree and runs the generic path), instead of one timeout per wait.
constexpr unsigned long long kScSpinTicks = 20000000ull;
__device__ __forceinline__ bool sc_give_up(int32_t *err, unsigned long long t0) {
  if (__hip_atomic_load(err + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return true;
  if (__builtin_amdgcn_s_memrealtime() - t0 > kScSpinTicks) {
    atomicAdd(err, 1);
    __hip_atomic_store(err + 5, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}

// Parity-mode draw offset of root b in simulation k: the sum of the depth flags of roots < b (the
// reference's single rand() stream, cnode.cpp:783-796). Wave-wide, in chunks of 256 roots (four flags per
// lane): sc_lookback_issue puts the first chunk's flags in flight, sc_lookback_finish spins (bounded, counted
// in err[0]) on the ones not yet published, then issues and sums every further chunk, and returns the
// wave-uniform sum. The late draw issues before the dynamics conv and finishes after it, so the cross-XCD
// round trip of the first chunk's loads overlaps the MFMAs. (B above the CU count: the grid is dispatched in
// block order, every root < 256 is resident from the start and a later root waits only on lower ones, which
// never wait on it: the waits end within one search.)
__device__ __forceinline__ void sc_lookback_issue(const ConvSearchArgs &p, int k, int b, unsigned long long epoch,
                                                  int lane, unsigned long long (&v)[4], int c0 = 0) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = c0 + 64 * u + lane;
    v[u] = q < b ? __hip_atomic_load(&p.flags[(size_t)k * p.B + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : (epoch << 32);
  }
}

__device__ __forceinline__ int sc_lookback_chunk(const ConvSearchArgs &p, int k, int b, unsigned long long epoch,
                                                  int lane, unsigned long long (&v)[4], int c0) {
  int base = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = c0 + 64 * u + lane;
    const unsigned long long t0 = (v[u] >> 32) != epoch ? __builtin_amdgcn_s_memrealtime() : 0ull;
    while ((v[u] >> 32) != epoch) {
      if (sc_give_up(p.err, t0)) {
        v[u] = epoch << 32;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v[u] = __hip_atomic_load(&p.flags[(size_t)k * p.B + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    base += (int)(v[u] & 0xffffffffu);
  }
  return base;
}

__device__ __forceinline__ int sc_lookback_finish(const ConvSearchArgs &p, int k, int b, unsigned long long epoch,
                                                  int lane, unsigned long long (&v)[4]) {
  int base = sc_lookback_chunk(p, k, b, epoch, lane, v, 0);
  if (b > 256) {  // wave-uniform; the common case (B <= 256) keeps the one-chunk straight line
    for (int c0 = 256; c0 < b; c0 += 256) {
      sc_lookback_issue(p, k, b, epoch, lane, v, c0);
      base += sc_lookback_chunk(p, k, b, epoch, lane, v, c0);
    }
  }
  return xor_sum(base);
}

__device__ __forceinline__ int sc_lookback(const ConvSearchArgs &p, int k, int b, unsigned long long epoch, int lane) {
  unsigned long long v[4];
  sc_lookback_issue(p, k, b, epoch, lane, v);
  return sc_lookback_finish(p, k, b, epoch, lane, v);
}

// this lane's 16 values of the dynamics conv's action map (the epilogue's order)
__device__ __forceinline__ void sc_load_amap(float4 (&am)[4], const float *actmap, int action, int c, int lane) {
  const float4 *amap = reinterpret_cast<const float4 *>(actmap + ((size_t)action * kCvCh + c) * kCvPix);
#pragma unroll
  for (int q = 0; q < 4; ++q) am[q] = amap[4 * q + (lane >> 4)];
}

// InverseScalarTransform's expectation of one support row by one wave (wave_support_expectation_reg
// arithmetic, the row read once) together with the row's raw sum for ensure_softmax's check
// (wave_row_sum's order).
template <int NPL>
__device__ __forceinline__ float sc_decode_row(const float *row, int V, float *raw_sum) {
  const int lane = threadIdx.x & 63;
  const float half = (float)((V - 1) / 2);
  float x[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int j = lane + 64 * q;
    x[q] = j < V ? row[j] : 0.0f;
  }
  float rs = 0.0f, mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < V) {
      rs += x[q];
      mx = fmaxf(mx, x[q]);
    }
  xor_sum_max(rs, mx);
  *raw_sum = rs;
  float e[NPL], sum = 0.0f;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    e[q] = lane + 64 * q < V ? expf(x[q] - mx) : 0.0f;
    if (lane + 64 * q < V) sum += e[q];
  }
  sum = xor_sum(sum);
  float acc = 0.0f;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < V) acc += (e[q] / sum) * ((float)(lane + 64 * q) - half);
  return xor_sum(acc);
}

// Output columns [jlo, jhi) of the three head layers (w2q [8][N2][4]: float4 k4 of column j at
// (k4 * N2 + j), so a wave-instruction reads 64 consecutive columns' float4s, 1 KiB contiguous), up to
// three columns per thread per round with every load of the round in flight; the FMA order of
// conv_heads_kernel (k = 0 .. 31 from zero, then + bias). Columns are independent, so any split of
// [0, N2) into ranges gives the same bits.
__device__ __forceinline__ void sc_head_out(const ConvSearchArgs &p, const float *lhid, float *llg, int N2, int jlo,
                                            int jhi, int tid) {
  for (int j0 = jlo; j0 < jhi; j0 += 3 * kScThreads) {
    float4 w2[3][8];
    float b2[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int j = min(j0 + u * kScThreads + tid, jhi - 1);
      const float4 *wc = reinterpret_cast<const float4 *>(p.w2q) + j;
#pragma unroll
      for (int q = 0; q < 8; ++q) w2[u][q] = wc[(size_t)q * N2];
      b2[u] = p.b2[j];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int j = j0 + u * kScThreads + tid;
      const float *hid = lhid + 32 * (j < p.Vr ? 0 : (j < p.Vr + p.Vv ? 1 : 2));
      float acc = 0.0f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 h4 = *reinterpret_cast<const float4 *>(hid + 4 * q);
        acc = __fmaf_rn(h4.x, w2[u][q].x, acc);
        acc = __fmaf_rn(h4.y, w2[u][q].y, acc);
        acc = __fmaf_rn(h4.z, w2[u][q].z, acc);
        acc = __fmaf_rn(h4.w, w2[u][q].w, acc);
      }
      if (j < jhi) llg[j] = acc + b2[u];
    }
  }
}

// Hidden layer of one head for this workgroup's env (conv_heads_kernel's arithmetic, same order):
// lane (part, c) sums its 128-wide K range with its 32 weight float4s (all loads in flight at once:
// one L2 round trip per head), the partial sums meet in K-part order, + bias, ReLU -> hid[c]. K is a
// multiple of 128 (lzm_search_conv checks). The weights are read through buffer resources (here and
// in sc_head_out1_rs): one 32-bit per-thread offset, the per-load constant in the scalar /
// immediate offset. With plain pointers the compiler
// hoisted one 64-bit address per load out of the simulation loop (24 per head) and, in the
// EfficientZero kernel, spilled them: every load then waited for a scratch reload (V/P hidden layers
// 40 K cycles per simulation instead of ~10 K). Same values, same FMA order, same bits.
__device__ __forceinline__ void sc_head_hidden_rs(const float *in, int K, const float *w1t, int head, float bias,
                                                  float *part, float *hid, int tid) {
  const int pt = tid >> 5, c = tid & 31;
  float acc = 0.0f;
  if (pt * 128 < K) {
    const float4 *x4 = reinterpret_cast<const float4 *>(in + pt * 128);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(w1t), 0, 3 * kHdParts * 32 * 32 * 16, 0x00020000);
    const int vo = (((head * kHdParts + pt) * 32) * 32 + c) * 16;
    float4 w1[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) w1[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, q * 512, 0));
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const float4 x = x4[q];
      acc = __fmaf_rn(x.x, w1[q].x, acc);
      acc = __fmaf_rn(x.y, w1[q].y, acc);
      acc = __fmaf_rn(x.z, w1[q].z, acc);
      acc = __fmaf_rn(x.w, w1[q].w, acc);
    }
  }
  part[pt * 32 + c] = acc;
  __syncthreads();
  if (tid < 32) {
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < kHdParts; ++q) s += part[q * 32 + tid];
    hid[tid] = fmaxf(s + bias, 0.0f);
  }
  __syncthreads();
}

// The first npin half-heads of w1t (half s: head s / 2, K steps 16 (s % 2) .. + 15 of every K part) copied
// into LDS once per launch: the head hidden layers' first half-head then reads LDS instead of joining the
// shared-rows L2 stream (§5.2 of DESIGN.md), and its exposed first round trip goes away.
__device__ __forceinline__ void sc_stage_wpin(float4 *pin, int npin, const float *w1t, int tid) {
  const float4 *w4 = reinterpret_cast<const float4 *>(w1t);
  for (int e = tid; e < npin * kHdParts * 16 * 32; e += kScThreads) {
    const int c = e & 31, q = (e >> 5) & 15, pt = (e >> 9) % kHdParts, s = (e >> 9) / kHdParts;
    pin[e] = w4[(((s >> 1) * kHdParts + pt) * 32 + 16 * (s & 1) + q) * 32 + c];
  }
}

// NH hidden layers (heads H0 .. H0 + NH - 1 of w1t) in one pass, sc_head_hidden's arithmetic and
// order for each head (same bits): the weights stream as 2 NH half-heads of 16 float4s per lane, the
// next half's loads in flight while the FMAs consume the current one, so the heads' L2 streams run
// back to back instead of one load-wait-reduce round each; one barrier pair for all of them.
// in[h] / K[h]: head H0 + h's input (LDS) and width; part: NH kHdParts 32 floats; hid[32 h + c].
// (Measured, Breakout one-launch search: the three hidden layers 14.9 K -> 12.7 K cycles per
// simulation.)
template <int NH, int H0>
__device__ __forceinline__ void sc_heads_hidden_rs(const float *const (&in)[NH], const int (&K)[NH], const float *w1t,
                                                   const float *b1, float *part, float *hid, int tid,
                                                   const float4 *pin = nullptr, int npin = 0) {
  const int pt = tid >> 5, c = tid & 31;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(w1t), 0, 3 * kHdParts * 32 * 32 * 16, 0x00020000);
  const int vo = ((pt * 32) * 32 + c) * 16;
  bool on[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) on[h] = pt * 128 < K[h];
  float4 wb[2][16];
  float acc[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) acc[h] = 0.0f;
  auto load = [&](int s, float4(&W)[16]) __attribute__((always_inline)) {
    const int h = s >> 1, half = s & 1;
    if (s < npin) {  // (uniform) the LDS copy, sc_stage_wpin's layout
      if (on[h]) {
#pragma unroll
        for (int q = 0; q < 16; ++q) W[q] = pin[((s * kHdParts + pt) * 16 + q) * 32 + c];
      }
    } else if (on[h]) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        W[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rs, vo, ((H0 + h) * kHdParts * 32 * 32 + (16 * half + q) * 32) * 16, 0));
    }
  };
  load(0, wb[0]);
#pragma unroll
  for (int s = 0; s < 2 * NH; ++s) {
    if (s + 1 < 2 * NH) load(s + 1, wb[(s + 1) & 1]);
    const int h = s >> 1, half = s & 1;
    if (on[h]) {
      const float4 *x4 = reinterpret_cast<const float4 *>(in[h] + pt * 128) + 16 * half;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 x = x4[q], w = wb[s & 1][q];
        acc[h] = __fmaf_rn(x.x, w.x, acc[h]);
        acc[h] = __fmaf_rn(x.y, w.y, acc[h]);
        acc[h] = __fmaf_rn(x.z, w.z, acc[h]);
        acc[h] = __fmaf_rn(x.w, w.w, acc[h]);
      }
    }
  }
#pragma unroll
  for (int h = 0; h < NH; ++h) part[(h * kHdParts + pt) * 32 + c] = acc[h];
  __syncthreads();
  if (tid < 32 * NH) {
    const int h = tid >> 5, cc = tid & 31;
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < kHdParts; ++q) s += part[(h * kHdParts + q) * 32 + cc];
    hid[tid] = fmaxf(s + b1[32 * H0 + tid], 0.0f);
  }
  __syncthreads();
}

// output columns [jlo, jhi), jhi - jlo <= kScThreads: one column per thread (sc_head_out's arithmetic)
__device__ __forceinline__ void sc_head_out1_rs(const ConvSearchArgs &p, const float *lhid, float *llg, int N2, int jlo,
                                                int jhi, int tid) {
  const int j = jlo + tid;
  if (j >= jhi) return;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.w2q), 0, N2 * 8 * 16, 0x00020000);
  float4 w2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) w2[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, j * 16, q * N2 * 16, 0));
  const float b2 = p.b2[j];
  const float *hid = lhid + 32 * (j < p.Vr ? 0 : (j < p.Vr + p.Vv ? 1 : 2));
  float acc = 0.0f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 h4 = *reinterpret_cast<const float4 *>(hid + 4 * q);
    acc = __fmaf_rn(h4.x, w2[q].x, acc);
    acc = __fmaf_rn(h4.y, w2[q].y, acc);
    acc = __fmaf_rn(h4.z, w2[q].z, acc);
    acc = __fmaf_rn(h4.w, w2[q].w, acc);
  }
  llg[j] = acc + b2;
}

// ensure_softmax + InverseScalarTransform of one decoded head by one wave (wave_support_expectation's
// arithmetic); returns h^-1 of the expectation (categorical) or of the raw value
__device__ __forceinline__ float sc_decode(const ConvSearchArgs &p, const float *row, int V) {
  float e;
  if (p.categorical) {
    float sm;
    e = V <= 128 ? sc_decode_row<2>(row, V, &sm) : V <= 640 ? sc_decode_row<10>(row, V, &sm) : sc_decode_row<16>(row, V, &sm);
    if ((threadIdx.x & 63) == 0 && fabsf(sm - 1.0f) <= 1e-5f + 1e-5f) atomicAdd(p.sdiag, 1);  // verdict undecidable
  } else {
    e = row[0];
  }
  return h_inverse(e);
}

// bounded spin of one lane on a 64-bit {epoch, payload} word (sc1 loads); returns the word (err[0]
// counts timeouts, the payload then reads 0)
__device__ __forceinline__ unsigned long long sc_wait_word(const unsigned long long *w, unsigned long long epoch,
                                                           int32_t *err) {
  unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = (v >> 32) != epoch ? __builtin_amdgcn_s_memrealtime() : 0ull;
  while ((v >> 32) != epoch) {
    if (sc_give_up(err, t0)) return epoch << 32;
    __builtin_amdgcn_s_sleep(1);
    v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return v;
}

template <int AHEAD, bool FAST, bool STAMPS = false>
__global__ __launch_bounds__(kScThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void search_conv_kernel(
    ConvSearchArgs p) {
  extern __shared__ uint4 sc_lds4[];
  uint16_t *act = reinterpret_cast<uint16_t *>(sc_lds4);
  float *smem = reinterpret_cast<float *>(sc_lds4);
  auto buf = [&](int i) { return act + i * kBxBuf; };
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = 16 * wv + (lane & 15);
  const int B = p.B, A = p.A, S = p.S;
  __shared__ uint32_t s_z0[31];
  __shared__ int s_players, s_epoch, s_x, s_act, s_vtp0, s_leafvtp, s_late, s_tlevel;
  __shared__ unsigned long long s_tmask;
  __shared__ int s_len[1];
  __shared__ float4 s_mm[1];
  __shared__ float s_dec[2];
  unsigned long long st_prev = 0, st_acc[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_w0 = 0;  // (the walk's own cycles, slot 10)
  const unsigned long long st_begin = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int n) {
    if (STAMPS && tid == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_acc[n] += now - st_prev;
      st_prev = now;
    }
  };

  // ---- stage root b's tree slice, the pUCT tables, seeds; zero the activation borders
  TreeView t;
  t.A = A; t.cap = p.cap; t.lut_n = p.lut_n; t.depth_cap = p.depth_cap; t.B = 1;
  NodeStat *ls = reinterpret_cast<NodeStat *>(smem + p.off_stat);
  NodeMeta *lm = reinterpret_cast<NodeMeta *>(smem + p.off_meta);
  float *lval = smem + p.off_val;
  float2 *llut = reinterpret_cast<float2 *>(smem + p.off_lut);
  int32_t *llegal = reinterpret_cast<int32_t *>(smem + p.off_legal);
  for (int e = tid; e < p.cap; e += kScThreads) {
    const NodeStat s = p.stat[(size_t)e * B + b];
    ls[e] = s;
    lm[e] = p.meta[(size_t)e * B + b];
    lval[e] = node_value(s);
  }
  for (int e = tid; e < p.lut_n; e += kScThreads) llut[e] = p.lut[e];
  for (int e = tid; e < A; e += kScThreads) llegal[e] = p.legal[(size_t)b * A + e];
  if (tid == 0) llegal[A] = p.nlegal[b];
  t.stat = ls; t.meta = lm; t.val = lval; t.lut = llut; t.legal = llegal; t.nlegal = llegal + A;
  t.pbt = nullptr;  // the walk divides (same bits) instead of a dependent table read: Breakout walk -3%
  t.path = reinterpret_cast<int32_t *>(smem + p.off_path);
  t.path_act = reinterpret_cast<int32_t *>(smem + p.off_pact);
  t.pathlen = s_len;
  uint32_t *s_seed = reinterpret_cast<uint32_t *>(smem + p.off_seed);
  uint32_t *s_pow = s_seed + S;
  if (p.step_count) {
    const long long cnt = *p.step_count;  // (read before the last workgroup's increment)
    for (int e = tid; e < S; e += kScThreads) s_seed[e] = (uint32_t)((p.step_base + cnt * (long long)S + e) % 1000000ll);
  } else {
    for (int e = tid; e < S; e += kScThreads) s_seed[e] = p.seeds[e];
  }
  if (!FAST && tid < 31) s_pow[tid] = p.pow16807[tid];
  bx_zero_borders(sc_lds4, tid, kScThreads);
  float4 *lpin = reinterpret_cast<float4 *>(smem + p.off_wpin);
  sc_stage_wpin(lpin, p.npin, p.w1t, tid);
  if (tid == 0) {
    s_mm[0] = p.step_fresh ? make_float4(kFloatMin, kFloatMax, p.step_delta, 0.0f) : p.minmax[b];
    s_vtp0 = p.vtp_in[b];
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {  // players (cnode.cpp:776-781), every load in flight at once
    int m = INT_MIN;
    for (int q = tid; q < B; q += 64) m = max(m, p.vtp_in[q]);
    m = xor_max(m);
    if (tid == 0) s_players = (m == -1) ? 1 : 2;
  }
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;
  float *lr = smem + p.off_r, *lhd = smem + p.off_hd, *lhid = smem + p.off_hid, *lpart = smem + p.off_part;
  float *llg = smem + p.off_lg;
  const int N2 = p.Vr + p.Vv + A;
  // trunk weights: this wave's stream of each 3x3 layer (lzm_conv.h bx layout), row scales and bounds
  const ConvTrunkLayout L = conv_trunk_layout_p(p.n_dres, p.n_pres, 1);
  const int n3 = 1 + 2 * p.n_dres + 2 * p.n_pres;
  const float *winv = p.w + L.sc;
  __shared__ float4 s_bd[kBxMaxLayers];  // the layers' bounds (staged below, before the first simulation's barrier)
  const float4 *wbd = s_bd;
  bx_stage_bounds(s_bd, p.w, L, n3 + 2, tid, kScThreads);
  auto layer_w = [&](int i) { return p.w + bx_layer_off(L, p.n_dres, i); };
  auto wave_stream = [&](const float *w) { return reinterpret_cast<const uint4 *>(w) + wv * 18 * kBxTerms * 64; };
  BxRing<AHEAD> ring;
  __shared__ uint32_t s_mx[4], s_wm[2][4];
  int range_bad = 0;
  float *lmax = smem + p.off_lmax;  // the exact max |x| of this root's pool latents, by slot (lzm_conv.h "Range")
  {  // slot 0: the root's latent
    float x0[16];
    const float *src = p.pool + (size_t)b * (kCvCh * kCvPix);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * q + 4 * (lane >> 4));
      x0[4 * q] = v.x; x0[4 * q + 1] = v.y; x0[4 * q + 2] = v.z; x0[4 * q + 3] = v.w;
    }
    const float m0 = bx_latent_max(x0, s_mx, wv, lane);
    if (tid == 0) lmax[0] = m0;  // (read after the first simulation's barriers)
  }

  for (int k = 0; k < S; ++k) {
    // ---- selection (wave 0; parity mode: draw-free walk, depth flag, look-back only for a value)
    // the dynamics conv's first weight chunks, in flight during the walk
    bx_prefetch<18, AHEAD, 0>(ring, wave_stream(p.w + L.dyn), lane);
    if (!FAST && tid < 31) seed_state_parallel(s_seed[k], s_pow, s_z0);
    __syncthreads();
    if (STAMPS && tid == 0) st_prev = __builtin_amdgcn_s_memtime();
    if (tid == 0) s_late = 0;
    if (wv == 0) {
      const float4 mm = s_mm[0];
      Descent d;
      if (STAMPS && tid == 0) st_w0 = __builtin_amdgcn_s_memtime();
      if (FAST) {
        const uint32_t seed = s_seed[k];
        auto draw = [seed, b](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)b, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        d = descend_wave<false, false, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
      } else {
        TieInfo ti;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        d = descend_wave<false, true, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, nodraw, &ti);
        if (STAMPS && tid == 0) {
          st_acc[10] += __builtin_amdgcn_s_memtime() - st_w0;
          st_acc[11] += d.len;              // levels walked (diagnostics)
          st_acc[12] += ti.status == 1 ? 1 : 0;  // late-draw ties
        }
        if (lane == 0 && ti.status != 2)
          __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        if (ti.status == 2) {
          // the depth depends on the draws: look back, walk with them, then publish
          const int base = sc_lookback(p, k, b, epoch, lane);
          const LaneDraws draw = lane_draws(p.coef, p.coef_positions, s_z0, base, 0, t.depth_cap, p.err + 1);
          d = descend_wave<false, false, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
          if (lane == 0)
            __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else if (ti.status == 1) {
          // a tie among unexpanded children: the leaf's parent (the latent to read) and the depth are
          // known, only the action waits for the draw — resolved after the dynamics conv's MFMAs
          // (late draw; issuing the flag loads here instead measured even: the wait is for the
          // predecessors to reach this simulation, not the loads' latency)
          if (lane == 0) {
            s_late = 1;
            s_tlevel = ti.level;
            s_tmask = ti.mask;
          }
        }
      }
      if (lane == 0) {
        s_x = d.x;
        s_act = d.action;
        s_len[0] = d.len;
        s_leafvtp = d.vtp;
        if (p.rec_x) {
          p.rec_x[(size_t)k * B + b] = d.x;
          p.rec_a[(size_t)k * B + b] = d.action;
          p.rec_len[(size_t)k * B + b] = d.len;
        }
      }
    }
    __syncthreads();
    stamp(0);
    // ---- trunk: the leaf's parent latent pool[x][b] and the action's map (registers; loads in flight
    // together), then the layers
    {
      const bool late = s_late != 0;
      const float *src = p.pool + ((size_t)max(s_x, 0) * B + b) * (kCvCh * kCvPix);
      float xres[16];
      float4 am[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * q + 4 * (lane >> 4));
        xres[4 * q] = v.x; xres[4 * q + 1] = v.y; xres[4 * q + 2] = v.z; xres[4 * q + 3] = v.w;
      }
      if (!late) sc_load_amap(am, p.actmap, s_act, c, lane);
      BxRange rg = bx_range_input(lmax[max(s_x, 0)]);
      {
        bxf4 in4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) in4[q] = bxf4{xres[4 * q], xres[4 * q + 1], xres[4 * q + 2], xres[4 * q + 3]};
        const float4 no_am[4] = {};
        bx_epilogue3<false>(in4, buf(0), 1.f, 0.f, false, no_am, xres, false, false, bx_pow2(rg.s_in), lane, c);
      }
      __syncthreads();
      stamp(1);
      for (int i = 0; i < n3; ++i) {
        const float *w = layer_w(i);
        const bool second = i > 0 && ((i - 1) & 1);  // a block's second conv: + residual, new block input
        const float bc = i ? w[kBx3Frag + c] : 0.f;
        const float4 bdi = wbd[i];
        const float wsc = winv[i * 64 + c];
        bxf4 acc[4];
        bx_conv<18, AHEAD, 0>(buf(i & 1), wave_stream(w), ring, lane, acc);
        if (i + 1 < n3) bx_prefetch<18, AHEAD, 0>(ring, wave_stream(layer_w(i + 1)), lane);
        if (i == 0 && late) {
          // late draw: the look-back and the tie's draw, then the action's map for the epilogue — by every
          // wave for itself (no barrier hands the action over); wave 0 files it. A spin timeout is counted
          // once per wave that met it and may leave the waves with different bases: any count invalidates
          // the search (lzm_check_errors raises), so such a latent is never used
          const unsigned long long lb0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
          const int base = sc_lookback(p, k, b, epoch, lane);
          if (STAMPS && tid == 0) st_acc[8] += __builtin_amdgcn_s_memtime() - lb0;
          const uint32_t rr = glibc_draw_wave(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.err + 1);
          unsigned long long m = s_tmask;
          int kk = (int)(rr % (uint32_t)__popcll(m));
          for (; kk > 0; --kk) m &= m - 1;
          const int jsel = __ffsll((long long)m) - 1;
          const int lvl = s_tlevel;
          const int parent = t.path[lvl];
          const int action = legal_at(t, 0, parent, jsel);
          if (tid == 0) {
            t.path_act[lvl] = action;
            t.path[lvl + 1] = 1 + A * t.meta[parent].latent + action;
            s_act = action;
            if (p.rec_a) p.rec_a[(size_t)k * B + b] = action;
          }
          sc_load_amap(am, p.actmap, action, c, lane);
        }
        const int s_out = bx_layer_scale(bdi, i == 0 || second, rg);
        bx_post_umax(s_wm[i & 1],
                     bx_epilogue3(acc, buf((i + 1) & 1), wsc * bx_pow2(-rg.s_in), bc, i == 0, am, xres,
                                  i == 0 || second, i == 0 || second, bx_pow2(s_out), lane, c),
                     wv, lane);
        __syncthreads();
        bx_range_take(rg, s_wm[i & 1], s_out);  // (the latent's max: filed)
        if (i == 2 * p.n_dres && tid == 0) lmax[k + 1] = rg.m_in;
        if (i == 2 * p.n_dres) {  // the next latent (registers, exact) and the reward planes
          float *dst = p.pool + ((size_t)(k + 1) * B + b) * (kCvCh * kCvPix) + c * kCvPix + 4 * (lane >> 4);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4 *>(dst + 16 * q) = float4{xres[4 * q], xres[4 * q + 1], xres[4 * q + 2], xres[4 * q + 3]};
          if (wv < 2)
            bx_conv1_layer<0>(buf((i + 1) & 1), p.w + L.rw, p.w + L.rb, winv + n3 * 64, bx_pow2(-rg.s_in), p.r_ch, lr,
                              lane, wv);
        }
      }
      if (wv < 2)
        bx_conv1_layer<0>(buf(n3 & 1), p.w + L.hw, p.w + L.hb, winv + (n3 + 1) * 64, bx_pow2(-rg.s_in), p.h_ch, lhd,
                          lane, wv);
      range_bad |= rg.bad;
    }
    __syncthreads();
    stamp(2);
    // ---- head MLPs: the three hidden layers
    {
      const float *const in[3] = {lr, lhd, lhd + p.off_policy};
      const int K[3] = {p.Kr, p.off_policy, p.Khd - p.off_policy};
      sc_heads_hidden_rs<3, 0>(in, K, p.w1t, p.b1, lpart, lhid, tid, lpin, p.npin);
    }
    stamp(3);
    // output columns (w2q [8][N2][4]: float4 k4 of column j at (k4 * N2 + j), so a wave-instruction
    // reads 64 consecutive columns' float4s, 1 KiB contiguous), up to three columns per thread per
    // round with every load of the round in flight; the FMA order of conv_heads_kernel (k = 0 .. 31
    // from zero, then + bias)
    for (int j0 = 0; j0 < N2; j0 += 3 * kScThreads) {
      float4 w2[3][8];
      float b2[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int j = min(j0 + u * kScThreads + tid, N2 - 1);
        const float4 *wc = reinterpret_cast<const float4 *>(p.w2q) + j;
#pragma unroll
        for (int q = 0; q < 8; ++q) w2[u][q] = wc[(size_t)q * N2];
        b2[u] = p.b2[j];
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int j = j0 + u * kScThreads + tid;
        const float *hid = lhid + 32 * (j < p.Vr ? 0 : (j < p.Vr + p.Vv ? 1 : 2));
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 h4 = *reinterpret_cast<const float4 *>(hid + 4 * q);
          acc = __fmaf_rn(h4.x, w2[u][q].x, acc);
          acc = __fmaf_rn(h4.y, w2[u][q].y, acc);
          acc = __fmaf_rn(h4.z, w2[u][q].z, acc);
          acc = __fmaf_rn(h4.w, w2[u][q].w, acc);
        }
        if (j < N2) llg[j] = acc + b2[u];
      }
    }
    __syncthreads();
    stamp(4);
    // ---- decode (wave 0 reward, wave 1 value), then expand + backup (wave 0)
    if (wv < 2) {
      const float *row = llg + (wv == 0 ? 0 : p.Vr);
      const int V = wv == 0 ? p.Vr : p.Vv;
      float e;
      if (p.categorical) {
        float sm;
        e = V <= 640 ? sc_decode_row<10>(row, V, &sm) : sc_decode_row<16>(row, V, &sm);
        if (lane == 0 && fabsf(sm - 1.0f) <= 1e-5f + 1e-5f) atomicAdd(p.sdiag, 1);  // batch verdict undecidable
      } else {
        e = row[0];
      }
      if (lane == 0) s_dec[wv] = h_inverse(e);
    }
    __syncthreads();
    stamp(5);
    if (wv == 0) {
      // wave 0 files the leaf's record and backs up while wave 1 initialises the leaf's children
      // (disjoint nodes, expand_wave's part argument)
      const float r = s_dec[0], v = s_dec[1];
      const int leaf = t.path[s_len[0]];
      const float *plg = llg + p.Vr + p.Vv;
      expand_wave(t, 0, leaf, s_leafvtp, k + 1, r, plg, -1, kExp2fTab, 1);
      backup_wave(t, 0, 0, 1, s_mm, s_leafvtp, v, p.disc);
      if (p.rec_dec) {
        if (lane < 2) p.rec_dec[((size_t)k * B + b) * 2 + lane] = lane ? v : r;
        if (lane < A) p.rec_logits[((size_t)k * B + b) * A + lane] = plg[lane];
      }
    } else if (wv == 1) {
      expand_wave(t, 0, 0, 0, k + 1, 0.0f, llg + p.Vr + p.Vv, -1, kExp2fTab, 2);
    }
    stamp(6);
  }
  __syncthreads();
  // ---- write back the slice (tree, last path, min-max)
  for (int e = tid; e < p.cap; e += kScThreads) {
    p.stat[(size_t)e * B + b] = ls[e];
    p.meta[(size_t)e * B + b] = lm[e];
  }
  for (int l = tid; l < p.depth_cap; l += kScThreads) {
    p.path[(size_t)l * B + b] = t.path[l];
    p.path_act[(size_t)l * B + b] = t.path_act[l];
  }
  if (STAMPS && tid == 0 && p.stamps) {
    st_acc[7] = __builtin_amdgcn_s_memtime() - st_begin;
    for (int n = 0; n < 13; ++n) atomicAdd(p.stamps + 40 + n, st_acc[n]);
  }
  // collect-step root outputs (root_outputs_kernel's values): visit counts per legal action, the root value
  if (p.out_dist && tid < A) {
    const int rl = lm[0].latent;
    p.out_dist[(size_t)b * A + tid] = (rl >= 0 && tid < llegal[A]) ? ls[1 + A * rl + llegal[tid]].visit : -1;
  }
  if (p.out_values && tid == 0) p.out_values[b] = node_value(ls[0]);
  if (tid == 0) {
    if (range_bad) atomicAdd(p.err + 4, 1);  // split activations out of the fp16 range (lzm_conv.h)
    p.minmax[b] = s_mm[0];
    p.pathlen[b] = s_len[0];
    // the last workgroup advances the epoch (no release fence: the kernel boundary orders the
    // write-back for every later reader) and the collect step's counter (every workgroup has read it)
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)gridDim.x - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.step_count && p.step_inc) *p.step_count += 1;
    }
  }
}


#ifndef LZM_EZ_POOL_AUX
#define LZM_EZ_POOL_AUX 16  // cache policy of the latent pool stores (16: sc1)
#endif
// The EfficientZero one-launch search (lzm_search_conv_ez). The grid is G = max(B, 2 T)
// workgroups; workgroup g owns root g (g < B) and K half (g & 1 or the XCD map below) of LSTM tile
// q(g) (g < 2 T). Per simulation, on top of the MuZero flow:
//   - the trunk writes root b's LSTM input row xin[b] = [reward planes | hpool[x][b]] with sc1 stores
//     and publishes {epoch, x, search_len} in xflags[k][b] (every storing wave's vmcnt(0), a barrier,
//     one agent-scope flag store: MI355X_MICROARCH.md's first hand-off row);
//   - the value / policy heads run while the other roots finish their trunks;
//   - the tile waits for its 64 rows' flags, runs the split-fp16 gate GEMM over its K half
//     (lp_tile_gemm, ez_lstm_gemm_cell_kernel's arithmetic), the upper half hands its partial sums to
//     the lower (pflags), which adds them, runs the cell with c0 = cpool[x][b] and files the masked c
//     state (its own slots: the tile map is fixed, so only this workgroup ever reads them), and hands
//     the unmasked h1 rows over (h1g, tflags);
//   - the root waits for its row's NB tiles, files the masked h state into hpool[k + 1][b] (read back
//     only by itself), and runs the value-prefix head on relu(BN(h1)), the decode, expand (is_reset =
//     search_len % horizon == 0) and the EfficientZero backup.
// Waits are only on events of the same simulation that precede the wait in every workgroup's
// program order, and every workgroup is resident (G <= CUs, one per CU), so the grid cannot deadlock;
// each spin is bounded and counted (err[0]).
template <int AHEAD, bool FAST, bool STAMPS = false>
__global__ __launch_bounds__(kScThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void search_conv_ez_kernel(
    ConvSearchArgs p) {
  extern __shared__ uint4 sc_lds4[];
  uint16_t *act = reinterpret_cast<uint16_t *>(sc_lds4);
  float *smem = reinterpret_cast<float *>(sc_lds4);
  auto buf = [&](int i) { return act + i * kBxBuf; };
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = 16 * wv + (lane & 15);
  const int B = p.B, A = p.A, S = p.S;
  const bool has_root = b < B;
  __shared__ uint32_t s_z0[31];
  __shared__ int s_players, s_epoch, s_x, s_act, s_vtp0, s_leafvtp, s_late, s_tlevel;
  __shared__ unsigned long long s_tmask;
  __shared__ int s_len[1];
  __shared__ float4 s_mm[1];
  __shared__ float s_dec[2];
  // STAMPS: [0] walk, [1] trunk input, [2] trunk layers, [3] value / policy hidden, [4] their outputs +
  // value decode, [5] LSTM tile, [6] value-prefix head, [7] expand + backup, [8] late look-back, [9] kernel,
  // [10] wait for the tile's rows, [11] wait for the upper K half, [12] wait for the row's tiles, [13] gate GEMM
  unsigned long long st_prev = 0, st_acc[14] = {};
  auto st_now = [&]() { return STAMPS ? __builtin_amdgcn_s_memtime() : 0ull; };
  const unsigned long long st_begin = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int n) {
    if (STAMPS && tid == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_acc[n] += now - st_prev;
      st_prev = now;
    }
  };

  // ---- stage root b's tree slice, the pUCT tables, seeds; zero the activation borders
  TreeView t;
  t.A = A; t.cap = p.cap; t.lut_n = p.lut_n; t.depth_cap = p.depth_cap; t.B = 1;
  NodeStat *ls = reinterpret_cast<NodeStat *>(smem + p.off_stat);
  NodeMeta *lm = reinterpret_cast<NodeMeta *>(smem + p.off_meta);
  float *lval = smem + p.off_val;
  float2 *llut = reinterpret_cast<float2 *>(smem + p.off_lut);
  int32_t *llegal = reinterpret_cast<int32_t *>(smem + p.off_legal);
  if (has_root) {
    for (int e = tid; e < p.cap; e += kScThreads) {
      const NodeStat s = p.stat[(size_t)e * B + b];
      ls[e] = s;
      lm[e] = p.meta[(size_t)e * B + b];
      lval[e] = node_value(s);
    }
    for (int e = tid; e < p.lut_n; e += kScThreads) llut[e] = p.lut[e];
    for (int e = tid; e < A; e += kScThreads) llegal[e] = p.legal[(size_t)b * A + e];
    if (tid == 0) llegal[A] = p.nlegal[b];
  }
  float *lpbt = smem + p.off_pbt;
  if (has_root) build_pbt(p.lut, p.pbt_rows, lpbt, tid, kScThreads);
  t.stat = ls; t.meta = lm; t.val = lval; t.lut = llut; t.legal = llegal; t.nlegal = llegal + A;
  t.pbt = p.pbt_rows ? lpbt : nullptr;
  t.path = reinterpret_cast<int32_t *>(smem + p.off_path);
  t.path_act = reinterpret_cast<int32_t *>(smem + p.off_pact);
  t.pathlen = s_len;
  uint32_t *s_seed = reinterpret_cast<uint32_t *>(smem + p.off_seed);
  uint32_t *s_pow = s_seed + S;
  if (p.step_count) {
    const long long cnt = *p.step_count;  // (read before the last workgroup's increment)
    for (int e = tid; e < S; e += kScThreads) s_seed[e] = (uint32_t)((p.step_base + cnt * (long long)S + e) % 1000000ll);
  } else {
    for (int e = tid; e < S; e += kScThreads) s_seed[e] = p.seeds[e];
  }
  if (!FAST && tid < 31) s_pow[tid] = p.pow16807[tid];
  if (tid == 0) {
    if (has_root) {
      s_mm[0] = p.step_fresh ? make_float4(kFloatMin, kFloatMax, p.step_delta, 0.0f) : p.minmax[b];
      s_vtp0 = p.vtp_in[b];
    }
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {  // players (cnode.cpp:776-781), every load in flight at once
    int m = INT_MIN;
    for (int q = tid; q < B; q += 64) m = max(m, p.vtp_in[q]);
    m = xor_max(m);
    if (tid == 0) s_players = (m == -1) ? 1 : 2;
  }
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;
  float *lr = smem + p.off_r, *lhd = smem + p.off_hd, *lhid = smem + p.off_hid, *lpart = smem + p.off_part;
  float *llg = smem + p.off_lg;
  const int N2 = p.Vr + p.Vv + A;

  // EfficientZero: this workgroup's LSTM tile (fixed for the launch)
  __shared__ int s_rx[64], s_rlen[64], s_rexp[64];
  const int T = p.T, NB = p.H / kLsUnits;
  const bool has_tile = b < 2 * T;
  int q = 0;
  LpTile tile{0, 0, 0};
  {
    int kh = b & 1;
    q = b >> 1;
    if ((T & 3) == 0) {
      // XCD map (block % 8 = XCD): one K half per XCD (XCD & 1) and consecutive tiles — whole
      // n-blocks, every row block — so an XCD's L2 holds its W slice (K / 2 x 64 columns per n-block)
      // and only its K half of the LSTM input rows; the split-K partner sits on the next XCD
      const int xcd = b & 7, j = b >> 3;
      q = (xcd >> 1) * (T >> 2) + j;
      kh = xcd & 1;
    }
    const int nb = q / p.nmb, mb = q - nb * p.nmb;
    tile = LpTile{kLsRows * mb, nb, kh};
  }
  const int Kx = p.Kx, H = p.H;
  typedef unsigned sc_u4 __attribute__((ext_vector_type(4)));

  // trunk weights: this wave's stream of each 3x3 layer (lzm_conv.h bx layout), row scales and bounds
  const ConvTrunkLayout L = conv_trunk_layout_p(p.n_dres, p.n_pres, 1);
  const int n3 = 1 + 2 * p.n_dres + 2 * p.n_pres;
  const float *winv = p.w + L.sc;
  __shared__ float4 s_bd[kBxMaxLayers];  // the layers' bounds (staged below, before the first simulation's barrier)
  const float4 *wbd = s_bd;
  bx_stage_bounds(s_bd, p.w, L, n3 + 2, tid, kScThreads);
  auto layer_w = [&](int i) { return p.w + bx_layer_off(L, p.n_dres, i); };
  auto wave_stream = [&](const float *w) { return reinterpret_cast<const uint4 *>(w) + wv * 18 * kBxTerms * 64; };
  BxRing<AHEAD> ring;
  __shared__ uint32_t s_mx[4], s_rmx[2], s_wm[2][4];
  int range_bad = 0;
  float *lmax = smem + p.off_lmax;  // the exact max |x| of this root's pool latents, by slot (lzm_conv.h "Range")
  if (has_root) {  // slot 0: the root's latent
    float x0[16];
    const float *src = p.pool + (size_t)b * (kCvCh * kCvPix);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * q + 4 * (lane >> 4));
      x0[4 * q] = v.x; x0[4 * q + 1] = v.y; x0[4 * q + 2] = v.z; x0[4 * q + 3] = v.w;
    }
    const float m0 = bx_latent_max(x0, s_mx, wv, lane);
    if (tid == 0) lmax[0] = m0;  // (read after the first simulation's barriers)
  }

  for (int k = 0; k < S; ++k) {
    if (has_root) {
      // ---- selection (wave 0; parity mode: draw-free walk, depth flag, look-back only for a value)
      // the dynamics conv's first weight chunks, in flight during the walk
      bx_prefetch<18, AHEAD, 0>(ring, wave_stream(p.w + L.dyn), lane);
      if (!FAST && tid < 31) seed_state_parallel(s_seed[k], s_pow, s_z0);
      bx_zero_borders(sc_lds4, tid, kScThreads);  // (every simulation: the LSTM stages reuse the buffers)
      __syncthreads();
      if (STAMPS && tid == 0) st_prev = __builtin_amdgcn_s_memtime();
      if (tid == 0) s_late = 0;
      if (wv == 0) {
        const float4 mm = s_mm[0];
        Descent d;
        if (FAST) {
          const uint32_t seed = s_seed[k];
          auto draw = [seed, b](int level) -> uint32_t {
            uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)b, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
            return o.x >> 1;
          };
          d = descend_wave<true, false, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
        } else {
          TieInfo ti;
          auto nodraw = [](int) -> uint32_t { return 0u; };
          d = descend_wave<true, true, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, nodraw, &ti);
          if (lane == 0 && ti.status != 2)
            __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          if (ti.status == 2) {
            // the depth depends on the draws: look back, walk with them, then publish
            const int base = sc_lookback(p, k, b, epoch, lane);
            const LaneDraws draw = lane_draws(p.coef, p.coef_positions, s_z0, base, 0, t.depth_cap, p.err + 1);
            d = descend_wave<true, false, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
            if (lane == 0)
              __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          } else if (ti.status == 1) {
            // a tie among unexpanded children: the leaf's parent (the latent to read) and the depth are
            // known, only the action waits for the draw — resolved after the dynamics conv's MFMAs
            // (late draw; issuing the flag loads here instead measured even: the wait is for the
            // predecessors to reach this simulation, not the loads' latency)
            if (lane == 0) {
              s_late = 1;
              s_tlevel = ti.level;
              s_tmask = ti.mask;
            }
          }
        }
        if (lane == 0) {
          s_x = d.x;
          s_act = d.action;
          s_len[0] = d.len;
          s_leafvtp = d.vtp;
          if (p.rec_x) {
            p.rec_x[(size_t)k * B + b] = d.x;
            p.rec_a[(size_t)k * B + b] = d.action;
            p.rec_len[(size_t)k * B + b] = d.len;
          }
        }
      }
      __syncthreads();
      stamp(0);
      // ---- trunk: the leaf's parent latent pool[x][b] and the action's map (registers; loads in flight
      // together), then the layers
      {
        const bool late = s_late != 0;
        const float *src = p.pool + ((size_t)max(s_x, 0) * B + b) * (kCvCh * kCvPix);
        float xres[16];
        float4 am[4];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * q4 + 4 * (lane >> 4));
          xres[4 * q4] = v.x; xres[4 * q4 + 1] = v.y; xres[4 * q4 + 2] = v.z; xres[4 * q4 + 3] = v.w;
        }
        if (!late) sc_load_amap(am, p.actmap, s_act, c, lane);
        {
          // the LSTM input row's hidden-state part: hpool[x][b] (this workgroup's own earlier writes, or
          // the roots' state) -> xin[b][r_ch * 64 ..] by sc1 stores
          if (tid < (H >> 2)) {
            const float4 v = reinterpret_cast<const float4 *>(p.hpool + ((size_t)max(s_x, 0) * B + b) * H)[tid];
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.xin + (size_t)b * Kx, 0, Kx * 4, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc_u4, v), rs, (Kx - H + 4 * tid) * 4, 0, 16);
          }
        }
        BxRange rg = bx_range_input(lmax[max(s_x, 0)]);
        {
          bxf4 in4[4];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) in4[q4] = bxf4{xres[4 * q4], xres[4 * q4 + 1], xres[4 * q4 + 2], xres[4 * q4 + 3]};
          const float4 no_am[4] = {};
          bx_epilogue3<false>(in4, buf(0), 1.f, 0.f, false, no_am, xres, false, false, bx_pow2(rg.s_in), lane, c);
        }
          __syncthreads();
        stamp(1);
        for (int i = 0; i < n3; ++i) {
          const float *w = layer_w(i);
          const bool second = i > 0 && ((i - 1) & 1);  // a block's second conv: + residual, new block input
          const float bc = i ? w[kBx3Frag + c] : 0.f;
          const float4 bdi = wbd[i];
          const float wsc = winv[i * 64 + c];
          bxf4 acc[4];
          bx_conv<18, AHEAD, 0>(buf(i & 1), wave_stream(w), ring, lane, acc);
          if (i + 1 < n3) bx_prefetch<18, AHEAD, 0>(ring, wave_stream(layer_w(i + 1)), lane);
          if (i == 0 && late) {
            // late draw: the look-back and the tie's draw, then the action's map for the epilogue — by every
            // wave for itself (no barrier hands the action over); wave 0 files it (a timeout: as in
            // search_conv_kernel, counted per wave, and it invalidates the search)
            const unsigned long long lb0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
            const int base = sc_lookback(p, k, b, epoch, lane);
            if (STAMPS && tid == 0) st_acc[8] += __builtin_amdgcn_s_memtime() - lb0;
            const uint32_t rr = glibc_draw_wave(p.coef, p.coef_positions, s_z0, base + s_tlevel, p.err + 1);
            unsigned long long m = s_tmask;
            int kk = (int)(rr % (uint32_t)__popcll(m));
            for (; kk > 0; --kk) m &= m - 1;
            const int jsel = __ffsll((long long)m) - 1;
            const int lvl = s_tlevel;
            const int parent = t.path[lvl];
            const int action = legal_at(t, 0, parent, jsel);
            if (tid == 0) {
              t.path_act[lvl] = action;
              t.path[lvl + 1] = 1 + A * t.meta[parent].latent + action;
              s_act = action;
              if (p.rec_a) p.rec_a[(size_t)k * B + b] = action;
            }
            sc_load_amap(am, p.actmap, action, c, lane);
          }
          const int s_out = bx_layer_scale(bdi, i == 0 || second, rg);
          bx_post_umax(s_wm[i & 1],
                       bx_epilogue3(acc, buf((i + 1) & 1), wsc * bx_pow2(-rg.s_in), bc, i == 0, am, xres,
                                    i == 0 || second, i == 0 || second, bx_pow2(s_out), lane, c),
                       wv, lane);
          __syncthreads();
          bx_range_take(rg, s_wm[i & 1], s_out);  // (the latent's max: filed)
          if (i == 2 * p.n_dres && tid == 0) lmax[k + 1] = rg.m_in;
          if (i == 2 * p.n_dres) {  // the next latent (registers, exact) and the reward planes
            // the latent by sc1 (write-through) stores, which do not keep the line in this XCD's L2: 16 KB
            // per root and simulation that would otherwise push the LSTM weights and the trunk's out of
            // it; read back (as a parent) at most once per later simulation
            const __amdgpu_buffer_rsrc_t lr4 = __builtin_amdgcn_make_buffer_rsrc(
                p.pool + ((size_t)(k + 1) * B + b) * (kCvCh * kCvPix), 0, kCvCh * kCvPix * 4, 0x00020000);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4)
              __builtin_amdgcn_raw_buffer_store_b128(
                  __builtin_bit_cast(sc_u4, float4{xres[4 * q4], xres[4 * q4 + 1], xres[4 * q4 + 2], xres[4 * q4 + 3]}),
                  lr4, (c * kCvPix + 4 * (lane >> 4) + 16 * q4) * 4, 0, LZM_EZ_POOL_AUX);
            if (wv < 2) {  // the reward planes: the LSTM input row's first part, sc1; their max for its scale
              const uint32_t rm = bx_conv1_layer<0, true>(buf((i + 1) & 1), p.w + L.rw, p.w + L.rb, winv + n3 * 64,
                                                          bx_pow2(-rg.s_in), p.r_ch, p.xin + (size_t)b * Kx, lane, wv);
              bx_post_max(s_rmx, rm, wv, lane);
            }
          }
        }
        if (wv < 2)
          bx_conv1_layer<0>(buf(n3 & 1), p.w + L.hw, p.w + L.hb, winv + (n3 + 1) * 64, bx_pow2(-rg.s_in), p.h_ch, lhd,
                            lane, wv);
        range_bad |= rg.bad;
      }
      // publish the LSTM input row: every storing wave drained, one barrier, one flag store
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {  // {epoch | row scale exponent + 128 : 8 | x : 12 | search_len : 12} (S <= 4094)
        const unsigned se = (unsigned)(ls_row_exp(__uint_as_float(max(s_rmx[0], s_rmx[1]))) + 128) & 0xffu;
        __hip_atomic_store(&p.xflags[(size_t)k * B + b],
                           (epoch << 32) | ((unsigned long long)se << 24) |
                               ((unsigned long long)(max(s_x, 0) & 0xfff) << 12) | (unsigned)(s_len[0] & 0xfff),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      stamp(2);
      // ---- head MLPs: value and policy now (while the other roots finish their trunks), the value
      // prefix after the LSTM
      sc_head_hidden_rs(lhd, p.off_policy, p.w1t, 1, tid < 32 ? p.b1[32 + tid] : 0.0f, lpart, lhid + 32, tid);
      sc_head_hidden_rs(lhd + p.off_policy, p.Khd - p.off_policy, p.w1t, 2, tid < 32 ? p.b1[64 + tid] : 0.0f, lpart,
                     lhid + 64, tid);
      stamp(3);
      if (N2 - p.Vr <= kScThreads)
        sc_head_out1_rs(p, lhid, llg, N2, p.Vr, N2, tid);
      else
        sc_head_out(p, lhid, llg, N2, p.Vr, N2, tid);
      __syncthreads();
      if (wv == 1) {
        const float v = sc_decode(p, llg + p.Vr, p.Vv);
        if (lane == 0) s_dec[1] = v;
      }
      stamp(4);
    }
    {
      // ---- the LSTM tile (gate GEMM over the tile's K half; the lower half runs the cell)
      if (has_tile) {
        const unsigned long long w0 = st_now();
        if (wv == 0) {  // the tile's rows: {x, search_len} from their flags
          const int row = tile.row0 + lane;
          unsigned long long v = 0;
          if (row < B) v = sc_wait_word(&p.xflags[(size_t)k * B + row], epoch, p.err);
          s_rx[lane] = (int)((v >> 12) & 0xfff);
          s_rlen[lane] = (int)(v & 0xfff);
          s_rexp[lane] = row < B ? (int)((v >> 24) & 0xff) - 128 : 0;
        }
        __syncthreads();
        const unsigned long long w1 = st_now();
        if (STAMPS && tid == 0) st_acc[10] += w1 - w0;
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(p.xin, 0, B * Kx * 4, 0x00020000);
        bxf4 acc[4];
        int lbad = 0;
        lp_tile_gemm(tile, B, Kx, xr, p.lwfrag, s_rexp, act, acc, lbad);
        range_bad |= lbad;
        if (STAMPS && tid == 0) st_acc[13] += st_now() - w1;
        const __amdgpu_buffer_rsrc_t pr =
            __builtin_amdgcn_make_buffer_rsrc(p.kpart + (size_t)q * (kLpThreads * 16), 0, kLpThreads * 16 * 4, 0x00020000);
        if (tile.kh == 1) {
          // upper K half: partial sums to the lower half (sc1 payload, drained, barrier, flag)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc_u4, acc[tt]), pr, (tid * 16 + 4 * tt) * 4, 0, 16);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0)
            __hip_atomic_store(&p.pflags[(size_t)k * T + q], (epoch << 32) | 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const int gate = lane & 3, ct = wv;
          const int unit = kLsUnits * tile.nb + 4 * ct + ((lane & 15) >> 2);
          // the cell's inputs (c0 from this workgroup's own state slots, or the roots' state)
          const float bias_l = p.lbias[(size_t)gate * H + unit], wsc = p.lwinv[(size_t)gate * H + unit];
          float c0[4], rsc[4][4];
          int rst[4];
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const int rl = 16 * tt + 4 * (lane >> 4) + gate, row = tile.row0 + rl;
            c0[tt] = 0.f;
            rst[tt] = 0;
            if (row < B) {
              c0[tt] = p.cpool[((size_t)s_rx[rl] * B + row) * H + unit];
              rst[tt] = p.horizon > 0 && (s_rlen[rl] % p.horizon) == 0;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)  // accumulator row 16 tt + 4 (lane >> 4) + r: 2^-(e_j + s_row)
              rsc[tt][r] = wsc * bx_pow2(-s_rexp[16 * tt + 4 * (lane >> 4) + r]);
          }
          const unsigned long long w2 = st_now();
          if (tid == 0) (void)sc_wait_word(&p.pflags[(size_t)k * T + q], epoch, p.err);
          __syncthreads();
          if (STAMPS && tid == 0) st_acc[11] += st_now() - w2;
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            acc[tt] += __builtin_bit_cast(bxf4, __builtin_amdgcn_raw_buffer_load_b128(pr, (tid * 16 + 4 * tt) * 4, 0, 16));
          // epilogue: + bias, the four gates of (row, unit) from the quad, the cell by lane gate = r
          // (ez_lstm_gemm_cell_kernel's operations in its order); h1 through LDS to whole 64-B rows
          float *s_h = smem;  // [64 rows][16 units] (the stage buffers are free after the barrier)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            float gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = __fmaf_rn(acc[tt][r], rsc[tt][r], bias_l);
              const float vi = ls_quad_bcast(v, 0), vf = ls_quad_bcast(v, 1), vg = ls_quad_bcast(v, 2), vo = ls_quad_bcast(v, 3);
              if (gate == r) { gi = vi; gf = vf; gg = vg; go = vo; }
            }
            const int rl = 16 * tt + 4 * (lane >> 4) + gate, row = tile.row0 + rl;
            const float cc = lstm_sigmoid(gf) * c0[tt] + lstm_sigmoid(gi) * tanhf(gg);
            const float hh = lstm_sigmoid(go) * tanhf(cc);
            s_h[rl * kLsUnits + (unit - kLsUnits * tile.nb)] = hh;
            if (row < B) p.cpool[((size_t)(k + 1) * B + row) * H + unit] = rst[tt] ? 0.0f : cc;
          }
          __syncthreads();
          {
            const int rl = tid >> 2, row = tile.row0 + rl;
            if (row < B) {
              const float4 v = reinterpret_cast<const float4 *>(s_h)[tid];
              const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(p.h1g, 0, B * H * 4, 0x00020000);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc_u4, v), hr,
                                                     (row * H + kLsUnits * tile.nb + 4 * (tid & 3)) * 4, 0, 16);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0)
            __hip_atomic_store(&p.tflags[(size_t)k * T + q], (epoch << 32) | 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      stamp(5);
      if (has_root) {
        // ---- the value-prefix head on this root's LSTM output: wait for the row's NB tiles (sc1 loads)
        const int mb = b / kLsRows;
        const unsigned long long w3 = st_now();
        if (wv == 0 && lane < NB) (void)sc_wait_word(&p.tflags[(size_t)k * T + lane * p.nmb + mb], epoch, p.err);
        if (wv == 1) {
          // meanwhile the leaf's expansion (everything but its value prefix, filed after the decode) and
          // best_action along the path (cnode.cpp:806)
          const int len = s_len[0];
          const int is_reset = (p.horizon > 0 && len % p.horizon == 0) ? 1 : 0;
          expand_wave(t, 0, t.path[len], s_leafvtp, k + 1, 0.0f, llg + p.Vr + p.Vv, is_reset);
          for (int l = lane; l < len; l += 64) t.meta[t.path[l]].best = t.path_act[l];
        }
        __syncthreads();
        if (STAMPS && tid == 0) st_acc[12] += st_now() - w3;
        const bool reset = p.horizon > 0 && (s_len[0] % p.horizon) == 0;
        if (tid < (H >> 2)) {
          const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(p.h1g + (size_t)b * H, 0, H * 4, 0x00020000);
          const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(hr, tid * 16, 0, 16));
          const float4 s4 = reinterpret_cast<const float4 *>(p.vp_s)[tid], t4 = reinterpret_cast<const float4 *>(p.vp_t)[tid];
          float4 x;
          x.x = fmaxf(__fmaf_rn(v.x, s4.x, t4.x), 0.0f);
          x.y = fmaxf(__fmaf_rn(v.y, s4.y, t4.y), 0.0f);
          x.z = fmaxf(__fmaf_rn(v.z, s4.z, t4.z), 0.0f);
          x.w = fmaxf(__fmaf_rn(v.w, s4.w, t4.w), 0.0f);
          reinterpret_cast<float4 *>(lr)[tid] = x;
          reinterpret_cast<float4 *>(p.hpool + ((size_t)(k + 1) * B + b) * H)[tid] =
              reset ? make_float4(0.f, 0.f, 0.f, 0.f) : v;
        }
        __syncthreads();
        sc_head_hidden_rs(lr, p.Kr, p.w1t, 0, tid < 32 ? p.b1[tid] : 0.0f, lpart, lhid, tid);
        if (p.Vr <= kScThreads)
          sc_head_out1_rs(p, lhid, llg, N2, 0, p.Vr, tid);
        else
          sc_head_out(p, lhid, llg, N2, 0, p.Vr, tid);
        __syncthreads();
        if (wv == 0) {
          const float r = sc_decode(p, llg, p.Vr);
          if (lane == 0) s_dec[0] = r;
        }
        __syncthreads();
        stamp(6);
      }
    }
    // ---- expand + backup (wave 0)
    if (has_root && wv == 0) {
      const float r = s_dec[0], v = s_dec[1];
      const int len = s_len[0];
      const int leaf = t.path[len];
      const float *plg = llg + p.Vr + p.Vv;
      const int is_reset = (p.horizon > 0 && len % p.horizon == 0) ? 1 : 0;
      if (lane == 0) t.stat[leaf].reward = r;  // the expansion's value prefix (expand_wave ran above)
      backup_wave_ez(t, 0, 0, 1, s_mm, s_leafvtp, v, p.disc);
      if (p.rec_reset && lane == 0) p.rec_reset[(size_t)k * B + b] = is_reset;
      if (p.rec_dec) {
        if (lane < 2) p.rec_dec[((size_t)k * B + b) * 2 + lane] = lane ? v : r;
        if (lane < A) p.rec_logits[((size_t)k * B + b) * A + lane] = plg[lane];
      }
    }
    stamp(7);
  }
  __syncthreads();
  // ---- write back the slice (tree, last path, min-max)
  if (has_root) {
    for (int e = tid; e < p.cap; e += kScThreads) {
      p.stat[(size_t)e * B + b] = ls[e];
      p.meta[(size_t)e * B + b] = lm[e];
    }
    for (int l = tid; l < p.depth_cap; l += kScThreads) {
      p.path[(size_t)l * B + b] = t.path[l];
      p.path_act[(size_t)l * B + b] = t.path_act[l];
    }
  }
  if (STAMPS && tid == 0 && p.stamps) {
    st_acc[9] = __builtin_amdgcn_s_memtime() - st_begin;
    for (int n = 0; n < 14; ++n) atomicAdd(p.stamps + 40 + n, st_acc[n]);
  }
  if (has_root && p.out_dist && tid < A) {  // collect-step root outputs, as the MuZero kernel
    const int rl = lm[0].latent;
    p.out_dist[(size_t)b * A + tid] = (rl >= 0 && tid < t.nlegal[0]) ? ls[1 + A * rl + t.legal[tid]].visit : -1;
  }
  if (has_root && p.out_values && tid == 0) p.out_values[b] = node_value(ls[0]);
  if (tid == 0) {
    if (range_bad) atomicAdd(p.err + 4, 1);  // split activations out of the fp16 range (lzm_conv.h, lzm_lstm.h)
    if (has_root) {
      p.minmax[b] = s_mm[0];
      p.pathlen[b] = s_len[0];
    }
    // the last workgroup advances the epoch (no release fence: the kernel boundary orders the
    // write-back for every later reader) and the collect step's counter
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)gridDim.x - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.step_count && p.step_inc) *p.step_count += 1;
    }
  }
}

}  // namespace lzm
