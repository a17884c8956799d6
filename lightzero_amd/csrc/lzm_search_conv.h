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
//   2. the four waves run the split-bf16 MFMA trunk (lzm_conv.h: dynamics conv + action map,
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
#include "lzm_search_mlp.h"
#include "lzm_tree.h"

namespace lzm {

constexpr int kScThreads = 256;

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
  // trunk (split-bf16 layout, lzm_conv_trunk_prepare_p) and heads (lzm_heads.h layouts)
  const float *w, *actmap;
  int n_dres, n_pres, r_ch, h_ch;
  const float *w1t, *b1, *w2c, *b2;  // w2c: the output layer column-major [N2][32] (16-B aligned)
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
  // dynamic LDS plan: float offsets (the two activation buffers come first)
  int off_stat, off_meta, off_val, off_lut, off_legal, off_path, off_pact, off_pbt, off_r, off_hd, off_hid, off_part,
      off_lg, off_seed;
};

// Hidden layer of one head for this workgroup's env (conv_heads_kernel's arithmetic, same order):
// lane (part, c) sums its 128-wide K range (32 float4 of weights, fetched in two halves of 16 to
// bound the registers), the partial sums meet in K-part order, + bias, ReLU -> hid[c].
__device__ __forceinline__ void sc_head_hidden(const float *in, int K, const float *w1t, int head, float bias,
                                               float *part, float *hid, int tid) {
  const int pt = tid >> 5, c = tid & 31;
  float acc = 0.0f;
  if (pt * 128 < K) {  // (K is a multiple of 128: lzm_search_conv checks)
    const float4 *x4 = reinterpret_cast<const float4 *>(in + pt * 128);
    const float4 *w = reinterpret_cast<const float4 *>(w1t) + ((size_t)(head * kHdParts + pt) * 32) * 32 + c;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // (a compiler barrier: keep the half's loads here rather than hoisted to the top of the kernel,
      // where every head's weights would be live at once)
      asm volatile("" ::: "memory");
      float4 w1[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w1[q] = w[(size_t)(16 * h + q) * 32];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k4 = 16 * h + q;
        const float4 x = x4[k4];
        acc = __fmaf_rn(x.x, w1[q].x, acc);
        acc = __fmaf_rn(x.y, w1[q].y, acc);
        acc = __fmaf_rn(x.z, w1[q].z, acc);
        acc = __fmaf_rn(x.w, w1[q].w, acc);
      }
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

template <int AHEAD, bool FAST>
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
  __shared__ int s_players, s_epoch, s_x, s_act, s_vtp0, s_leafvtp;
  __shared__ int s_len[1];
  __shared__ float4 s_mm[1];
  __shared__ float s_dec[2];

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
  float *lpbt = smem + p.off_pbt;
  build_pbt(p.lut, p.pbt_rows, lpbt, tid, kScThreads);
  t.stat = ls; t.meta = lm; t.val = lval; t.lut = llut; t.legal = llegal; t.nlegal = llegal + A;
  t.pbt = p.pbt_rows ? lpbt : nullptr;
  t.path = reinterpret_cast<int32_t *>(smem + p.off_path);
  t.path_act = reinterpret_cast<int32_t *>(smem + p.off_pact);
  t.pathlen = s_len;
  uint32_t *s_seed = reinterpret_cast<uint32_t *>(smem + p.off_seed);
  uint32_t *s_pow = s_seed + S;
  for (int e = tid; e < S; e += kScThreads) s_seed[e] = p.seeds[e];
  if (!FAST && tid < 31) s_pow[tid] = p.pow16807[tid];
  for (int k = tid; k < 2 * 3 * 36 * 8; k += kScThreads) {  // [buffer][term][border position][16-B chunk]
    const int ch = k & 7, bp = (k >> 3) % 36, plane = k / (36 * 8);
    const int ps = bp < 10 ? bp : bp < 20 ? 80 + bp : (1 + ((bp - 20) >> 1)) * 10 + ((bp - 20) & 1) * 9;
    sc_lds4[(plane * kBxComp + ps * 64) / 8 + ch] = uint4{0u, 0u, 0u, 0u};
  }
  if (tid == 0) {
    s_mm[0] = p.minmax[b];
    s_vtp0 = p.vtp_in[b];
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {  // players (cnode.cpp:776-781), every load in flight at once
    int m = INT_MIN;
    for (int q = tid; q < B; q += 64) m = max(m, p.vtp_in[q]);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) m = max(m, __shfl_xor(m, d, 64));
    if (tid == 0) s_players = (m == -1) ? 1 : 2;
  }
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;
  float *lr = smem + p.off_r, *lhd = smem + p.off_hd, *lhid = smem + p.off_hid, *lpart = smem + p.off_part;
  float *llg = smem + p.off_lg;
  const int N2 = p.Vr + p.Vv + A;

  // trunk weights: this wave's stream of each 3x3 layer (lzm_conv.h bx layout)
  const ConvTrunkLayout L = conv_trunk_layout_p(p.n_dres, p.n_pres, 1);
  const int n3 = 1 + 2 * p.n_dres + 2 * p.n_pres;
  auto layer_w = [&](int i) { return p.w + bx_layer_off(L, p.n_dres, i); };
  auto wave_stream = [&](const float *w) { return reinterpret_cast<const uint4 *>(w) + wv * 18 * 3 * 64; };
  BxRing<AHEAD> ring;

  for (int k = 0; k < S; ++k) {
    // ---- selection (wave 0; parity mode: draw-free walk, depth flag, look-back only for a value)
    if (!FAST && tid < 31) seed_state_parallel(s_seed[k], s_pow, s_z0);
    __syncthreads();
    if (wv == 0) {
      const float4 mm = s_mm[0];
      Descent d;
      if (FAST) {
        const uint32_t seed = s_seed[k];
        auto draw = [seed, b](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)b, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        d = descend_wave<false, false>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
      } else {
        TieInfo ti;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        d = descend_wave<false, true>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, nodraw, &ti);
        if (lane == 0 && ti.status != 2)
          __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        if (ti.status != 0) {
          int base = 0;
          for (int q = lane; q < b; q += 64) {
            unsigned long long v;
            long long spins = 0;
            while (true) {
              v = __hip_atomic_load(&p.flags[(size_t)k * B + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if ((v >> 32) == epoch) break;
              if (++spins > (1ll << 22)) {
                atomicAdd(p.err, 1);
                v = 0;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            base += (int)(v & 0xffffffffu);
          }
#pragma unroll
          for (int s = 32; s > 0; s >>= 1) base += __shfl_xor(base, s, 64);
          const uint32_t *coef = p.coef;
          const int npos = p.coef_positions;
          int32_t *ovf = p.err + 1;
          if (ti.status == 1) {
            // a tie among unexpanded children: the draw picks the leaf, the depth stays
            const uint32_t rr = glibc_draw(coef, npos, s_z0, base + ti.level, ovf);
            unsigned long long m = ti.mask;
            int kk = (int)(rr % (uint32_t)__popcll(m));
            for (; kk > 0; --kk) m &= m - 1;
            const int jsel = __ffsll((long long)m) - 1;
            const int parent = t.path[ti.level];
            const int action = legal_at(t, 0, parent, jsel);
            const int leaf = 1 + A * t.meta[parent].latent + action;
            if (lane == 0) {
              t.path_act[ti.level] = action;
              t.path[ti.level + 1] = leaf;
            }
            d.action = action;
            d.leaf = leaf;
          } else {
            // the depth depends on the draws: walk with them, then publish
            auto draw = [coef, npos, ovf, base](int level) -> uint32_t {
              return glibc_draw(coef, npos, s_z0, base + level, ovf);
            };
            d = descend_wave<false, false>(t, 0, 0, 1, mm, players, s_vtp0, p.disc, draw, nullptr);
            if (lane == 0)
              __hip_atomic_store(&p.flags[(size_t)k * B + b], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
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
    // ---- trunk: the dynamics conv's first weight chunks, the leaf's parent latent pool[x][b] and the
    // action's map (registers; all loads in flight together), then the layers
    {
      bx_prefetch<18, AHEAD, 0>(ring, wave_stream(p.w + L.dyn), lane);
      const float *src = p.pool + ((size_t)max(s_x, 0) * B + b) * (kCvCh * kCvPix);
      float xres[16];
      float4 am[4];
      const float4 *amap = reinterpret_cast<const float4 *>(p.actmap + ((size_t)s_act * kCvCh + c) * kCvPix);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * q + 4 * (lane >> 4));
        xres[4 * q] = v.x; xres[4 * q + 1] = v.y; xres[4 * q + 2] = v.z; xres[4 * q + 3] = v.w;
        am[q] = amap[4 * q + (lane >> 4)];
      }
      {
        bxf4 in4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) in4[q] = bxf4{xres[4 * q], xres[4 * q + 1], xres[4 * q + 2], xres[4 * q + 3]};
        const float4 no_am[4] = {};
        bx_epilogue3<0, 4, false>(in4, buf(0), 0.f, false, no_am, xres, false, false, lane, c);
      }
      __syncthreads();
      for (int i = 0; i < n3; ++i) {
        const float *w = layer_w(i);
        const bool second = i > 0 && ((i - 1) & 1);  // a block's second conv: + residual, new block input
        const float bc = i ? w[kBx3Frag + c] : 0.f;
        bxf4 acc[4];
        bx_conv<18, AHEAD, 0>(buf(i & 1), wave_stream(w), ring, lane, acc);
        if (i + 1 < n3) bx_prefetch<18, AHEAD, 0>(ring, wave_stream(layer_w(i + 1)), lane);
        bx_epilogue3(acc, buf((i + 1) & 1), bc, i == 0, am, xres, i == 0 || second, i == 0 || second, lane, c);
        __syncthreads();
        if (i == 2 * p.n_dres) {  // the next latent (registers, exact) and the reward planes
          float *dst = p.pool + ((size_t)(k + 1) * B + b) * (kCvCh * kCvPix) + c * kCvPix + 4 * (lane >> 4);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4 *>(dst + 16 * q) = float4{xres[4 * q], xres[4 * q + 1], xres[4 * q + 2], xres[4 * q + 3]};
          if (wv < 2) bx_conv1_layer<0>(buf((i + 1) & 1), p.w + L.rw, p.w + L.rb, p.r_ch, lr, lane, wv);
        }
      }
      if (wv < 2) bx_conv1_layer<0>(buf(n3 & 1), p.w + L.hw, p.w + L.hb, p.h_ch, lhd, lane, wv);
      __syncthreads();
    }
    // ---- head MLPs (conv_heads_kernel's arithmetic): hidden layers, then the output columns
    sc_head_hidden(lr, p.Kr, p.w1t, 0, tid < 32 ? p.b1[tid] : 0.0f, lpart, lhid, tid);
    sc_head_hidden(lhd, p.off_policy, p.w1t, 1, tid < 32 ? p.b1[32 + tid] : 0.0f, lpart, lhid + 32, tid);
    sc_head_hidden(lhd + p.off_policy, p.Khd - p.off_policy, p.w1t, 2, tid < 32 ? p.b1[64 + tid] : 0.0f, lpart,
                   lhid + 64, tid);
    // output columns: column-major weights (w2c [N2][32], 8 contiguous float4 per column), one column
    // per thread per round; the FMA order of conv_heads_kernel (k = 0 .. 31 from zero, then + bias)
    for (int j = tid; j < N2; j += kScThreads) {
      const float4 *wc = reinterpret_cast<const float4 *>(p.w2c) + (size_t)j * 8;
      float4 w2[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) w2[q] = wc[q];
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
    __syncthreads();
    // ---- decode (wave 0 reward, wave 1 value), then expand + backup (wave 0)
    if (wv < 2) {
      const float *row = llg + (wv == 0 ? 0 : p.Vr);
      const int V = wv == 0 ? p.Vr : p.Vv;
      float e;
      if (p.categorical) {
        const float sm = wave_row_sum(row, V);
        if (lane == 0 && fabsf(sm - 1.0f) <= 1e-5f + 1e-5f) atomicAdd(p.sdiag, 1);  // batch verdict undecidable
        e = wave_support_expectation(row, V, true);
      } else {
        e = row[0];
      }
      if (lane == 0) s_dec[wv] = h_inverse(e);
    }
    __syncthreads();
    if (wv == 0) {
      const float r = s_dec[0], v = s_dec[1];
      const int leaf = t.path[s_len[0]];
      const float *plg = llg + p.Vr + p.Vv;
      expand_wave(t, 0, leaf, s_leafvtp, k + 1, r, plg);
      backup_wave(t, 0, 0, 1, s_mm, s_leafvtp, v, p.disc);
      if (p.rec_dec) {
        if (lane < 2) p.rec_dec[((size_t)k * B + b) * 2 + lane] = lane ? v : r;
        if (lane < A) p.rec_logits[((size_t)k * B + b) * A + lane] = plg[lane];
      }
    }
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
  if (tid == 0) {
    p.minmax[b] = s_mm[0];
    p.pathlen[b] = s_len[0];
    // the last workgroup advances the epoch (no release fence: the kernel boundary orders the
    // write-back for every later reader)
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == (uint32_t)gridDim.x - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace lzm
