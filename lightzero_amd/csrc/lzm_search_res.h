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

// Resident weight layout (lzm_mlp_prepare writes it after the generic kernel layout; res_source
// below is its definition). Every block is [slot][lane] float4, so a wave-instruction of a block
// is one contiguous 1 KiB read.
//   D (128 x 128, six of them): slot j, lane l: W[64 (l & 1) + 4 j .. +3][l >> 1]
//   RH (128 -> 32 reward head hidden): slot j < 4: W[16 (l & 7) + 4 j ..][l >> 3]
//   VPH (128 -> 64: [value hidden | policy hidden]): slot j < 8: W[32 (l & 3) + 4 j ..][l >> 2]
//   S (32 -> 601 support head): slots 0-7: column l, k = 4 j; slots 8-15: column 256 + l;
//      slots 16-19: column 512 + (l >> 1), k = 16 (l & 1) + 4 (j - 16), lanes < 2 * kRTail
//   PO (32 -> A policy output): one slot: W[4 (l & 7) ..][l >> 3], l >> 3 < A
// then the biases ([6][128] D, [32] RH, [64] VPH, [604] RS, [604] VS, [32] PO) and the one-hot
// action rows of fc_dynamics[0], [A][128].
struct ResNet {
  const float4 *d[6];  // fc_dynamics[0] (latent rows), fc_dynamics[1], fc_dynamics_2[0..1], fc_prediction_common[0..1]
  const float4 *rh, *vph, *rs, *vs, *po;
  const float *bd, *brh, *bvph, *brs, *bvs, *bpo, *act;
  // LDS float offsets beyond SearchArgs' tree plan
  int off_x0, off_t1, off_nl, off_t2, off_t3, off_rh, off_hv, off_lg, off_act, off_wd1, off_wd2;
};

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
    *layer = src[b]; *col = l >> 1; *k = 64 * (l & 1) + 4 * j + e;
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
template <int NS>
__device__ __forceinline__ void res_fetch(const float4 *blk, float4 *dst) {
  const __amdgpu_buffer_rsrc_t r = wave_rsrc(blk, NS * kRT * 16);
  const int vo = (int)threadIdx.x * 16;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, j * kRT * 16, 0);
    dst[j] = make_float4(v.x, v.y, v.z, v.w);
  }
}

// Partial dot product of 4*NJ consecutive inputs x4[0..NJ) with weights w(j): four independent
// FMA chains (k mod 4), summed as (c0 + c1) + (c2 + c3).
template <int NJ, typename WF>
__device__ __forceinline__ float dot4(const float4 *x4, WF w) {
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float4 v = x4[j];
    const float4 q = w(j);
    a0 = __fmaf_rn(v.x, q.x, a0);
    a1 = __fmaf_rn(v.y, q.y, a1);
    a2 = __fmaf_rn(v.z, q.z, a2);
    a3 = __fmaf_rn(v.w, q.w, a3);
  }
  return (a0 + a1) + (a2 + a3);
}

// Full pre-activation of this lane's column of a 128 x 128 layer (both lanes of a pair get it).
template <typename WF>
__device__ __forceinline__ float dense128(const float *x, WF w) {
  const float h = dot4<16>(reinterpret_cast<const float4 *>(x) + 16 * (threadIdx.x & 1), w);
  return h + dpp_f<0xB1>(h);
}

// Logits of one support head (input: 32 floats in LDS; weights: the 20-slot buffer P): lane l
// gets columns l, 256 + l and (l < 2 * kRTail, l even) 512 + (l >> 1).
__device__ __forceinline__ void support_logits(const float *h, const float4 *P, float b0, float b1, float b2,
                                               float &z0, float &z1, float &z2) {
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  z0 = dot4<8>(h4, [&](int j) { return P[j]; }) + b0;
  z1 = dot4<8>(h4, [&](int j) { return P[8 + j]; }) + b1;
  const float t = dot4<4>(h4 + 4 * (threadIdx.x & 1), [&](int j) { return P[16 + j]; });
  z2 = (t + dpp_f<0xB1>(t)) + b2;
}

// Support expectation + h^-1 (scaling_transform.py:118-128) over the workgroup; every wave returns
// the same value. red: 12 floats of LDS owned by this call site. Two barriers.
__device__ __forceinline__ float support_decode(float z0, float z1, float z2, float *red) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool v2 = tid < 2 * kRTail && !(tid & 1);
  float m = fmaxf(z0, z1);
  if (v2) m = fmaxf(m, z2);
  m = wave_max_dpp(m);
  if (lane == 0) red[wid] = m;
  __syncthreads();
  const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float half = (float)((kRV - 1) / 2);
  const float e0 = expf(z0 - M), e1 = expf(z1 - M), e2 = v2 ? expf(z2 - M) : 0.0f;
  float se = (e0 + e1) + e2;
  float sj = (e0 * ((float)tid - half) + e1 * ((float)(kRT + tid) - half)) + e2 * ((float)(2 * kRT + (tid >> 1)) - half);
  se = wave_sum(se);
  sj = wave_sum(sj);
  if (lane == 0) {
    red[4 + wid] = se;
    red[8 + wid] = sj;
  }
  __syncthreads();
  const float SE = (red[4] + red[5]) + (red[6] + red[7]);
  const float SJ = (red[8] + red[9]) + (red[10] + red[11]);
  return h_inverse(SJ / SE);
}

// Sum of the draw counts published by workgroups < g for simulation k (wave-wide; bounded spin).
__device__ inline int lookback_sum(const SearchArgs &p, int k, int g, int G, unsigned long long epoch) {
  const int lane = threadIdx.x & 63;
  int sum = 0;
  for (int q = lane; q < g; q += 64) {
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
  return sum;
}

__global__ __launch_bounds__(kRT) __attribute__((amdgpu_waves_per_eu(1, 1))) void search_res_kernel(SearchArgs p, ResNet n) {
  extern __shared__ float4 smem4[];
  float *smem = reinterpret_cast<float *>(smem4);
  const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x, lane = tid & 63, wid = tid >> 6;
  const int B = p.B, A = p.A;
  const int i = g;  // one root per workgroup
  unsigned long long stamp_ = p.phase ? __builtin_amdgcn_s_memtime() : 0ull;

  __shared__ uint32_t s_z0[31];
  __shared__ int s_players, s_epoch, s_x, s_act, s_status, s_tlevel, s_vtp;
  __shared__ int s_len[1];
  __shared__ unsigned long long s_tmask;
  __shared__ float4 s_mm;
  __shared__ float s_red[24];
  __shared__ unsigned long long s_phase[64];
  if (p.phase && tid < 64) s_phase[tid] = 0ull;

  // ---- tree slice into LDS (node records, value cache, pUCT tables, legal list, path)
  TreeView t;
  t.A = A; t.cap = p.cap; t.lut_n = p.lut_n; t.depth_cap = p.depth_cap; t.B = 1;
  t.path = reinterpret_cast<int32_t *>(smem + p.off_path);
  t.path_act = reinterpret_cast<int32_t *>(smem + p.off_pact);
  t.pathlen = s_len;
  {
    NodeStat *ls = reinterpret_cast<NodeStat *>(smem + p.off_stat);
    NodeMeta *lm = reinterpret_cast<NodeMeta *>(smem + p.off_meta);
    float2 *llut = reinterpret_cast<float2 *>(smem + p.off_lut);
    int32_t *llegal = reinterpret_cast<int32_t *>(smem + p.off_legal);
    float *lval = smem + p.off_val;
    for (int e = tid; e < p.cap; e += kRT) {
      const NodeStat s = p.stat[(size_t)e * B + i];
      ls[e] = s;
      lm[e] = p.meta[(size_t)e * B + i];
      lval[e] = node_value(s);
    }
    for (int e = tid; e < p.lut_n; e += kRT) llut[e] = p.lut[e];
    float *lpbt = smem + p.off_pbt;
    for (int r = 0; r < p.pbt_rows; ++r) {
      const float y = p.lut[r].y;
      for (int v = tid; v <= r; v += kRT) lpbt[r * (r + 1) / 2 + v] = y / (float)(v + 1);
    }
    for (int e = tid; e < A; e += kRT) llegal[e] = p.legal[(size_t)i * A + e];
    if (tid == 0) llegal[A] = p.nlegal[i];
    t.stat = ls; t.meta = lm; t.lut = llut; t.legal = llegal; t.nlegal = llegal + A; t.val = lval;
    t.pbt = p.pbt_rows ? lpbt : nullptr;
  }
  if (tid == 0) {
    s_mm = p.minmax[i];
    s_vtp = p.vtp_in[i];
    int m = INT_MIN;
    for (int q = 0; q < B; ++q) m = max(m, p.vtp_in[q]);
    s_players = (m == -1) ? 1 : 2;
    s_epoch = (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t *s_seeds = reinterpret_cast<uint32_t *>(smem + p.off_misc);
  uint32_t *s_pow = s_seeds + p.S;
  for (int e = tid; e < p.S; e += kRT) s_seeds[e] = p.seeds[e];
  if (!p.fast)
    for (int e = tid; e < 31; e += kRT) s_pow[e] = p.pow16807[e];

  // ---- network residency: LDS layers, action rows, register layers and biases
  float *X0 = smem + n.off_x0, *T1 = smem + n.off_t1, *NL = smem + n.off_nl, *T2 = smem + n.off_t2,
        *T3 = smem + n.off_t3, *RHo = smem + n.off_rh, *HV = smem + n.off_hv, *LG = smem + n.off_lg,
        *ACT = smem + n.off_act;
  const float4 *WD1 = reinterpret_cast<const float4 *>(smem + n.off_wd1);
  const float4 *WD2 = reinterpret_cast<const float4 *>(smem + n.off_wd2);
  for (int e = tid; e < kRSlotsD * kRT; e += kRT) {
    reinterpret_cast<float4 *>(smem + n.off_wd1)[e] = n.d[1][e];
    reinterpret_cast<float4 *>(smem + n.off_wd2)[e] = n.d[2][e];
  }
  for (int e = tid; e < A * kRHid; e += kRT) ACT[e] = n.act[e];
  float4 wD3[kRSlotsD], wD4[kRSlotsD], wD5[kRSlotsD], wRH[kRSlotsRH], wVPH[kRSlotsVPH], wPO[1];
  res_fetch<kRSlotsD>(n.d[3], wD3);
  res_fetch<kRSlotsD>(n.d[4], wD4);
  res_fetch<kRSlotsD>(n.d[5], wD5);
  res_fetch<kRSlotsRH>(n.rh, wRH);
  res_fetch<kRSlotsVPH>(n.vph, wVPH);
  res_fetch<kRSlotsPO>(n.po, wPO);
  const int cD = tid >> 1, pD = tid & 1, cRH = tid >> 3, pRH = tid & 7, cVP = tid >> 2, pVP = tid & 3, cPO = tid >> 3;
  float bD[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) bD[q] = n.bd[q * kRHid + cD];
  const float bRH = n.brh[cRH], bVP = n.bvph[cVP], bPO = cPO < A ? n.bpo[cPO] : 0.0f;
  const int ct = 2 * kRT + (tid >> 1);
  const float bRS0 = n.brs[tid], bRS1 = n.brs[kRT + tid], bRS2 = tid < 2 * kRTail ? n.brs[ct] : 0.0f;
  const float bVS0 = n.bvs[tid], bVS1 = n.bvs[kRT + tid], bVS2 = tid < 2 * kRTail ? n.bvs[ct] : 0.0f;
  // the streamed buffer: fc_dynamics[0] for the first simulation
  float4 P[kRSlotsS];
  res_fetch<kRSlotsD>(n.d[0], P);
#pragma unroll
  for (int j = kRSlotsD; j < kRSlotsS; ++j) P[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  __syncthreads();
  const int players = s_players;
  const unsigned long long epoch = (unsigned long long)(uint32_t)s_epoch;
  LZM_STAMP(10);

  for (int k = 0; k < p.S; ++k) {
    const uint32_t seed = s_seeds[k];
    if (!p.fast) seed_state_parallel(seed, s_pow, s_z0);
    // ---- selection (wave 0, one lane per child): descend_wave, lzm_tree.h
    if (wid == 0) {
      const float4 mm = s_mm;
      if (p.fast) {
        auto draw = [seed, i](int level) -> uint32_t {
          uint4 o = philox4x32_10(make_uint4((uint32_t)level, (uint32_t)i, 0u, 0u), make_uint2(seed, 0x4c5a4d43u));
          return o.x >> 1;
        };
        Descent d = descend_wave<false, false>(t, 0, 0, 1, mm, players, s_vtp, p.disc, draw, nullptr);
        if (lane == 0) { s_len[0] = d.len; s_x = d.x; s_act = d.action; s_status = 0; }
      } else {
        TieInfo ti;
        auto nodraw = [](int) -> uint32_t { return 0u; };
        Descent d = descend_wave<false, true>(t, 0, 0, 1, mm, players, s_vtp, p.disc, nodraw, &ti);
        if (lane == 0) {
          s_len[0] = d.len; s_x = d.x; s_act = d.action;
          s_status = ti.status; s_tlevel = ti.level; s_tmask = ti.mask;
          // publish this root's draw count at once (its depth is known unless status 2)
          if (ti.status != 2)
            __hip_atomic_store(&p.flags[(size_t)k * G + g], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    LZM_STAMP(0);
    const int status = s_status;
    if (status == 2) {
      // the depth depends on a draw: look back now, then walk with the draws (exact semantics)
      if (wid == 0) {
        const int base = lookback_sum(p, k, g, G, epoch);
        if (lane == 0) {
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
    // ---- gather the leaf's parent latent: X0 = pool[x][i]
    if (tid < kRHid / 4)
      reinterpret_cast<float4 *>(X0)[tid] =
          reinterpret_cast<const float4 *>(p.pool + ((size_t)max(s_x, 0) * B + i) * kRHid)[tid];
    __syncthreads();
    LZM_STAMP(2);
    // ---- fc_dynamics[0], latent rows (streamed weights in P)
    const float z0 = dense128(X0, [&](int j) { return P[j]; });
    if (status == 1) {
      // a tie among unexpanded children: the draw picks the action (the latent is known)
      if (wid == 0) {
        const int base = lookback_sum(p, k, g, G, epoch);
        if (lane == 0) {
          const int lvl = s_tlevel;
          const uint32_t rr = glibc_draw(p.coef, p.coef_positions, s_z0, base + lvl, p.diag);
          unsigned long long m = s_tmask;
          int kk = (int)(rr % (uint32_t)__popcll(m));
          for (; kk > 0; --kk) m &= m - 1;
          const int jsel = __ffsll((long long)m) - 1;
          const int parent = t.path[lvl];
          const int action = legal_at(t, 0, parent, jsel);
          t.path_act[lvl] = action;
          t.path[lvl + 1] = 1 + A * t.meta[parent].latent + action;
          s_act = action;
        }
      }
      __syncthreads();
    }
    res_fetch<kRSlotsS>(n.rs, P);  // the reward support head, five steps on
    const int act = s_act;
    if (p.rec_x && tid == 0) {
      p.rec_x[(size_t)k * B + i] = s_x;
      p.rec_a[(size_t)k * B + i] = act;
      p.rec_len[(size_t)k * B + i] = s_len[0];
    }
    // + the action's one-hot row, bias, ReLU (muzero_model_mlp.py:188-190)
    if (pD == 0) T1[cD] = fmaxf((z0 + ACT[act * kRHid + cD]) + bD[0], 0.0f);
    __syncthreads();
    // ---- fc_dynamics[1] (LDS weights) + latent residual -> next latent
    {
      const float z = dense128(T1, [&](int j) { return WD1[j * kRT + tid]; });
      if (pD == 0) NL[cD] = fmaxf(z + bD[1], 0.0f) + X0[cD];
    }
    __syncthreads();
    LZM_STAMP(3);
    // file the next latent (mcts_ctree.py:305): pool[k + 1][i]
    if (tid < kRHid / 4)
      reinterpret_cast<float4 *>(p.pool + ((size_t)(k + 1) * B + i) * kRHid)[tid] = reinterpret_cast<const float4 *>(NL)[tid];
    // ---- fc_dynamics_2 (LDS, registers) -> reward head hidden -> reward support, decoded
    {
      const float z = dense128(NL, [&](int j) { return WD2[j * kRT + tid]; });
      if (pD == 0) T2[cD] = fmaxf(z + bD[2], 0.0f);
    }
    __syncthreads();
    {
      const float z = dense128(T2, [&](int j) { return wD3[j]; });
      if (pD == 0) T3[cD] = fmaxf(z + bD[3], 0.0f);
    }
    __syncthreads();
    {
      float h = dot4<kRSlotsRH>(reinterpret_cast<const float4 *>(T3) + 4 * pRH, [&](int j) { return wRH[j]; });
      h += dpp_f<0xB1>(h);
      h += dpp_f<0x4E>(h);
      h += dpp_f<0x141>(h);
      if (pRH == 0) RHo[cRH] = fmaxf(h + bRH, 0.0f);
    }
    __syncthreads();
    float rdec;
    {
      float a0, a1, a2;
      support_logits(RHo, P, bRS0, bRS1, bRS2, a0, a1, a2);
      res_fetch<kRSlotsS>(n.vs, P);  // the value support head, four steps on
      rdec = support_decode(a0, a1, a2, s_red);
    }
    LZM_STAMP(4);
    // ---- prediction trunk (registers) on the next latent
    {
      const float z = dense128(NL, [&](int j) { return wD4[j]; });
      if (pD == 0) T2[cD] = fmaxf(z + bD[4], 0.0f);
    }
    __syncthreads();
    {
      const float z = dense128(T2, [&](int j) { return wD5[j]; });
      if (pD == 0) T3[cD] = fmaxf(z + bD[5], 0.0f);
    }
    __syncthreads();
    LZM_STAMP(5);
    // ---- [value | policy] head hidden, then value support (decoded) and policy logits
    {
      float h = dot4<kRSlotsVPH>(reinterpret_cast<const float4 *>(T3) + 8 * pVP, [&](int j) { return wVPH[j]; });
      h += dpp_f<0xB1>(h);
      h += dpp_f<0x4E>(h);
      if (pVP == 0) HV[cVP] = fmaxf(h + bVP, 0.0f);
    }
    __syncthreads();
    float vdec;
    {
      const float4 hp = reinterpret_cast<const float4 *>(HV + kRF)[tid & 7];
      float q = __fmaf_rn(hp.x, wPO[0].x, 0.0f);
      q = __fmaf_rn(hp.y, wPO[0].y, q);
      q = __fmaf_rn(hp.z, wPO[0].z, q);
      q = __fmaf_rn(hp.w, wPO[0].w, q);
      q += dpp_f<0xB1>(q);
      q += dpp_f<0x4E>(q);
      q += dpp_f<0x141>(q);
      if ((tid & 7) == 0 && cPO < A) LG[cPO] = q + bPO;
      float a0, a1, a2;
      support_logits(HV, P, bVS0, bVS1, bVS2, a0, a1, a2);
      res_fetch<kRSlotsD>(n.d[0], P);  // fc_dynamics[0] for the next simulation
      vdec = support_decode(a0, a1, a2, s_red + 12);
    }
    LZM_STAMP(6);
    if (p.rec_dec && tid == 0) {
      p.rec_dec[((size_t)k * B + i) * 2] = rdec;
      p.rec_dec[((size_t)k * B + i) * 2 + 1] = vdec;
      for (int a = 0; a < A; ++a) p.rec_logits[((size_t)k * B + i) * A + a] = LG[a];
    }
    // ---- expand + backup (cbatch_backpropagate, cnode.cpp:480-500), wave 0
    if (wid == 0) {
      const int len = s_len[0];
      const int leaf = t.path[len];
      int vtp = s_vtp;
      if (players > 1)
        for (int l = 0; l < len; ++l) vtp = (vtp == 1) ? 2 : 1;
      expand_wave(t, 0, leaf, vtp, k + 1, rdec, LG);
      backup_wave(t, 0, 0, 1, &s_mm, vtp, vdec, p.disc);
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
  __syncthreads();
  if (p.phase && tid < 64 && s_phase[tid]) atomicAdd(p.phase + tid, s_phase[tid]);
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
