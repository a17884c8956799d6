// lzm_traverse_lb.h — parity-mode batch_traverse over many workgroups (generic search path).
//
// cbatch_traverse (lzero/mcts/ctree/ctree_muzero/lib/cnode.cpp:755-824; EfficientZero
// ctree_efficientzero/lib/cnode.cpp:756-814) walks the roots in order while drawing one rand()
// per tree level from ONE process-wide glibc stream, so root i's draws start at the sum of the
// depths of roots < i. traverse_glibc_kernel honours that in one workgroup by iterating the
// offsets to their fixed point. Here every root gets its own wave, as in the fused search
// (lzm_search_mlp.h): the walk first runs draw-free (descend_wave CLASSIFY: a tie among
// unexpanded children ends the walk at the same depth whichever child wins), the root publishes
// its depth in a 64-bit {epoch, count} word at once, and only a root that needs a draw VALUE
// sums its predecessors' words (decoupled look-back) and evaluates its draws straight from the
// seeded state through the coefficient table (random_r is linear over Z/2^32). A root whose depth
// depends on a draw (a tie reaching an expanded child) publishes after walking with its draws.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_search_mlp.h"
#include "lzm_tree.h"

namespace lzm {

constexpr int kTlbThreads = 256;  // four roots per workgroup, one wave each

struct TraverseLbArgs {
  TreeView t;
  const float4 *minmax;
  const uint32_t *seed;
  const int32_t *vtp_in;
  int32_t *out_x, *out_y, *out_a, *out_vtp, *out_len;
  long long *out_a64;
  float disc;
  const uint32_t *coef;  // [coef_positions][31]
  int coef_positions;
  const uint32_t *pow16807;   // [31]
  unsigned long long *flags;  // [B] {epoch, depth}
  uint32_t *epoch;            // [2] epoch, done counter
  int32_t *diag;              // [0] passes (1)
  int32_t *err;               // sticky error counters (lzm_check_errors): [0] look-back spin timeouts,
                              // [1] draw positions beyond the coefficient table
  const int32_t *reuse_action;  // optional [B] ReZero true actions (search-with-reuse), with
  const float *reuse_value;     // [B] their reuse values; null: plain search
  unsigned long long *stamps;   // LZM_PHASE_TIMING (diagnostic instantiation): per-phase shader cycles
                                // summed over roots and launches: [32] setup, [33] draw-free walk,
                                // [34] look-back + draw, [35] outputs, [36] roots, [37] roots needing
                                // a draw, [38] max kernel-start -> root-done
};

// Workgroup-level part of a look-back traverse (every thread calls it): the seeded glibc state and
// the launch epoch in LDS. Returns the epoch; *players = the batch's player count.
__device__ inline unsigned long long traverse_lb_setup(const TraverseLbArgs &p, uint32_t *s_z0, uint32_t *s_pow,
                                                       int *s_epoch, int *players) {
  // every global read of the setup in one round (seed, 16807 powers, epoch, the batch's to_play
  // values for the player count), then one barrier: players = (max(virtual_to_play) == -1) ? 1 : 2
  // (cnode.cpp:776-781) from per-wave maxima
  __shared__ int s_wmax[16];
  const int tid = threadIdx.x, lane = tid & 63, nw = blockDim.x >> 6;
  const uint32_t seed = *p.seed;
  const uint32_t pw = tid < 31 ? p.pow16807[tid] : 0u;
  const int ep = tid == 0 ? (int)__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  int m = INT_MIN;
  for (int q = tid; q < p.t.B; q += blockDim.x) m = max(m, p.vtp_in[q]);
  m = xor_max(m);
  if (lane == 0) s_wmax[tid >> 6] = m;
  if (tid < 31) s_pow[tid] = pw;
  if (tid == 0) *s_epoch = ep;
  __syncthreads();
  int mx = s_wmax[0];
  for (int w = 1; w < nw; ++w) mx = max(mx, s_wmax[w]);
  *players = mx == -1 ? 1 : 2;
  seed_state_parallel(seed, s_pow, s_z0);
  __syncthreads();
  return (unsigned long long)(uint32_t)*s_epoch;
}

// One root's walk by one wave (all 64 lanes): draw-free classification, depth published at once,
// look-back only when a draw value is needed (see the header comment).
template <bool EZ, bool STAMPS = false>
__device__ inline void traverse_lb_root(const TraverseLbArgs &p, int i, const uint32_t *s_z0, unsigned long long epoch,
                                        int players, unsigned long long t0 = 0, unsigned long long t1 = 0) {
  const TreeView &t = p.t;
  const int lane = threadIdx.x & 63, B = t.B;
  const float4 mm = p.minmax[i];
  const int vtp0 = p.vtp_in[i];
  TieInfo ti;
  auto nodraw = [](int) -> uint32_t { return 0u; };
  const int ta = p.reuse_action ? p.reuse_action[i] : -1;
  const float rv = p.reuse_action ? p.reuse_value[i] : 0.0f;
  Descent d = descend_wave<EZ, true, true>(t, i, i, B, mm, players, vtp0, p.disc, nodraw, &ti, ta, rv);
  const unsigned long long t2 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  if (lane == 0 && ti.status != 2)
    __hip_atomic_store(&p.flags[i], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ti.status != 0) {
    // draw offset: the depths of every earlier root (wave-wide look-back, bounded spin)
    int base = 0;
    for (int q = lane; q < i; q += 64) {
      unsigned long long v;
      long long spins = 0;
      while (true) {
        v = __hip_atomic_load(&p.flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    base = xor_sum(base);
    const uint32_t *coef = p.coef;
    const int npos = p.coef_positions;
    int32_t *diag = p.err + 1;
    if (ti.status == 1) {
      // a tie among unexpanded children: the draw picks the leaf, the depth stays
      const uint32_t rr = glibc_draw(coef, npos, s_z0, base + ti.level, diag);
      unsigned long long m = ti.mask;
      int kk = (int)(rr % (uint32_t)__popcll(m));
      for (; kk > 0; --kk) m &= m - 1;
      const int jsel = __ffsll((long long)m) - 1;
      const int parent = t.path[(size_t)ti.level * B + i];
      const int action = legal_at(t, i, parent, jsel);
      if (lane == 0) {
        t.path_act[(size_t)ti.level * B + i] = action;
        t.path[(size_t)(ti.level + 1) * B + i] = 1 + t.A * t.meta[nidx(t, parent, i)].latent + action;
      }
      d.action = action;
      d.leaf = 1 + t.A * t.meta[nidx(t, parent, i)].latent + action;
    } else {
      // the depth depends on the draws: walk with them, then publish
      const LaneDraws draw = lane_draws(coef, npos, s_z0, base, 0, t.depth_cap, diag);
      d = descend_wave<EZ, false, true>(t, i, i, B, mm, players, vtp0, p.disc, draw, nullptr, ta, rv);
      if (lane == 0)
        __hip_atomic_store(&p.flags[i], (epoch << 32) | (unsigned)d.len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const unsigned long long t3 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  if (lane == 0) {
    p.out_x[i] = d.x;
    p.out_y[i] = i;
    p.out_a[i] = d.action;
    if (p.out_a64) p.out_a64[i] = d.action;
    p.out_vtp[i] = d.vtp;
    p.out_len[i] = d.len;
    t.pathlen[i] = d.len;
  }
  // best_action along the final path (cnode.cpp:806)
  for (int l = lane; l < d.len; l += 64) {
    const int node = t.path[(size_t)l * B + i];
    t.meta[nidx(t, node, i)].best = t.path_act[(size_t)l * B + i];
  }
  if (STAMPS && lane == 0 && p.stamps) {
    const unsigned long long t4 = __builtin_amdgcn_s_memtime();
    atomicAdd(p.stamps + 32, t1 - t0);
    atomicAdd(p.stamps + 33, t2 - t1);
    atomicAdd(p.stamps + 34, t3 - t2);
    atomicAdd(p.stamps + 35, t4 - t3);
    atomicAdd(p.stamps + 36, 1ull);
    if (ti.status != 0) atomicAdd(p.stamps + 37, 1ull);
    atomicMax(p.stamps + 38, t4 - t0);
  }
}

// The last workgroup to finish advances the epoch for the next launch (every thread calls it). No
// release fence: nothing inside the launch reads data behind this counter (the draw counts travel
// in the atomic flag words; the kernel boundary orders everything else), and on gfx950 an
// agent-scope release is an L2 writeback (buffer_wbl2) per workgroup.
__device__ inline void traverse_lb_finish(const TraverseLbArgs &p, unsigned long long epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) p.diag[0] = 1;
    const uint32_t done = atomicAdd(p.epoch + 1, 1u);
    if (done == gridDim.x - 1) {
      p.epoch[1] = 0;
      __hip_atomic_store(p.epoch, (uint32_t)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// W waves (roots) per workgroup
template <bool EZ, int W = kTlbThreads / 64, bool STAMPS = false>
__global__ __launch_bounds__(64 * W) void traverse_lookback_kernel(TraverseLbArgs p) {
  __shared__ uint32_t s_z0[31], s_pow[31];
  __shared__ int s_epoch;
  int players;
  const unsigned long long t0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  const unsigned long long epoch = traverse_lb_setup(p, s_z0, s_pow, &s_epoch, &players);
  const unsigned long long t1 = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  const int i = blockIdx.x * W + (threadIdx.x >> 6);
  if (i < p.t.B) traverse_lb_root<EZ, STAMPS>(p, i, s_z0, epoch, players, t0, t1);
  traverse_lb_finish(p, epoch);
}

}  // namespace lzm
