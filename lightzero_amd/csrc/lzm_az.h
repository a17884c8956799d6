// lzm_az.h — batched AlphaZero tree search for TicTacToe on the device.
//
// The reference searches one board at a time, on the host, with a Python callback per simulation
// (lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp:47-254, node_alphazero.h). Here B boards are
// searched together: per simulation ONE launch finishes the previous simulation (expand the leaf with
// the network's priors, or score the terminal position; update_recursive with alternating signs) and
// runs the next descent, writing the leaf's network input (current_state / 2) for the batched
// policy-value call that follows. The descent replays the TicTacToe moves on the group's registers
// (the simulate env of the reference), so no env object exists on either side.
//
// Mapping: a 16-lane group per board, lane = action (cells 0..8). The pUCT score of child `a` is the
// reference's double expression with the glibc `log` term and `sqrt` of the parent count taken from
// host-built tables over the integer count (lut_pb, lut_sqrt), so the scores are bit-identical; the
// arg-max is a 4-step xor butterfly that keeps the lowest action on ties (first strict maximum in
// std::map order). Node fields keep the reference types: prior / value_sum float, visit int.
//
// Tree layout in HBM (SoA, one row of `cap` = 1 + 9 (S + 1) nodes per board, children of a node
// contiguous in action order): visit, vsum, prior, first (-1 = leaf), nch, act.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_numerics.h"

namespace lzm {

constexpr int kAzCells = 9;
constexpr int kAzGroup = 16;
constexpr int kAzPath = 10;      // root + at most 9 moves
constexpr int kAzThreads = 64;   // 4 boards per workgroup: B = 512 -> 128 workgroups

struct AzTree {
  int B, S, cap;
  int32_t *visit;       // [B][cap]
  float *vsum;          // [B][cap]
  float *prior;         // [B][cap]
  int32_t *first;       // [B][cap] index of the first child, -1 while a leaf
  int32_t *nch;         // [B][cap]
  int32_t *act;         // [B][cap] action that leads to the node
  int32_t *nnodes;      // [B]
  int32_t *root_board;  // [B][9] 0 empty, 1 / 2 stones
  int32_t *root_player; // [B] player to move at the root (1 / 2)
  int32_t *path;        // [B][kAzPath] node indices of the current descent
  int32_t *leaf;        // [B][4] depth, done, winner, player to move at the leaf
  int32_t *leaf_board;  // [B][9]
  double *lut_pb;       // [S + 1] log((n + base + 1) / base) + init   (glibc, host-built)
  double *lut_sqrt;     // [S + 1] sqrt(n)
  double *noise;        // [9][9] row n-1: the reference's default-seeded Dirichlet vector for n children
};

struct AzStepArgs {
  int sim;              // -1: expand the roots; k >= 0: finish simulation k
  int with_noise;
  double noise_weight;
  const float *probs;   // [B][pstride] policy probabilities of the evaluated positions
  int pstride;
  const float *values;  // [B] (element stride vstride)
  int vstride;
  float *state;         // [B][3][3][3] network input of the next positions to evaluate
};

// get_done_winner_cython.pyx, scanned in the same order (cell-major, 4 directions)
__device__ inline void az_done_winner(const int *bd, int &done, int &winner) {
  const int di[4] = {1, 1, 1, 0}, dj[4] = {-1, 0, 1, 1};
  bool has_legal = false;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const int p = bd[i * 3 + j];
      if (p == 0) {
        has_legal = true;
        continue;
      }
      const int d0 = j > 0 ? 0 : 1, d1 = j < 2 ? 4 : 3;
      for (int d = d0; d < d1; ++d) {
        int x = i, y = j, count = 0;
        for (int k = 0; k < 3; ++k) {
          if (x < 0 || x >= 3 || y < 0 || y >= 3 || bd[x * 3 + y] != p) break;
          x += di[d];
          y += dj[d];
          if (++count == 3) {
            done = 1;
            winner = p;
            return;
          }
        }
      }
    }
  done = has_legal ? 0 : 1;
  winner = -1;
}

// current_state()[1] of the reference env (tictactoe_env.py:350-376) for the player to move
__device__ inline void az_write_state(float *st, int l, int cell, int player) {
  if (l >= kAzCells) return;
  st[l] = cell == player ? 0.5f : 0.0f;
  st[kAzCells + l] = cell == 3 - player ? 0.5f : 0.0f;
  st[2 * kAzCells + l] = 0.5f * (float)player;
}

__device__ inline uint32_t az_group_mask(bool pred, int gbase) {
  return (uint32_t)((__ballot(pred) >> gbase) & 0xffffull);
}

// _expand_leaf_node: one child per empty cell (action order), prior = float(probs[a]); at the root,
// optionally _add_exploration_noise: float(double(prior) * (1 - w) + noise[i] * w)
__device__ inline void az_expand(const AzTree &t, size_t nb, int b, int node, int base, int l, int gbase, int cell,
                                 float pr, bool noise, double w) {
  const bool legal = l < kAzCells && cell == 0;
  const uint32_t gm = az_group_mask(legal, gbase);
  const int n = __popc(gm);
  const int rank = __popc(gm & ((1u << l) - 1u));
  if (legal) {
    const size_t c = nb + base + rank;
    float p = pr;
    if (noise) p = (float)((double)pr * (1.0 - w) + t.noise[(n - 1) * kAzCells + rank] * w);
    t.visit[c] = 0;
    t.vsum[c] = 0.0f;
    t.prior[c] = p;
    t.first[c] = -1;
    t.nch[c] = 0;
    t.act[c] = l;
  }
  if (l == 0) {
    t.first[nb + node] = n > 0 ? base : -1;
    t.nch[nb + node] = n;
    t.nnodes[b] = base + n;
  }
}

__global__ void __launch_bounds__(kAzThreads) az_begin_kernel(AzTree t, const int32_t *boards,
                                                              const int32_t *start_index, float *state) {
  const int b = blockIdx.x * (kAzThreads / kAzGroup) + threadIdx.x / kAzGroup;
  const int l = threadIdx.x & (kAzGroup - 1);
  if (b >= t.B) return;
  const int player = start_index[b] == 0 ? 1 : 2;  // players[start_player_index]
  const int cell = l < kAzCells ? boards[(size_t)b * kAzCells + l] : 0;
  if (l < kAzCells) t.root_board[(size_t)b * kAzCells + l] = cell;
  if (l == 0) t.root_player[b] = player;
  az_write_state(state + (size_t)b * 27, l, cell, player);
}

__global__ void __launch_bounds__(kAzThreads) az_step_kernel(AzTree t, AzStepArgs a) {
  const int b = blockIdx.x * (kAzThreads / kAzGroup) + threadIdx.x / kAzGroup;
  const int l = threadIdx.x & (kAzGroup - 1);
  const int gbase = (threadIdx.x & 63) & ~(kAzGroup - 1);
  if (b >= t.B) return;  // group-uniform
  const size_t nb = (size_t)b * t.cap;
  int32_t *path = t.path + (size_t)b * kAzPath;
  const float pr = l < kAzCells ? a.probs[(size_t)b * a.pstride + l] : 0.0f;
  if (a.sim < 0) {
    // a fresh root (Node()), expanded with the root evaluation; noise only when sampling
    const int cell = l < kAzCells ? t.root_board[(size_t)b * kAzCells + l] : -1;
    if (l == 0) {
      t.visit[nb] = 0;
      t.vsum[nb] = 0.0f;
      t.prior[nb] = 1.0f;
      t.act[nb] = -1;
    }
    az_expand(t, nb, b, 0, 1, l, gbase, cell, pr, a.with_noise != 0, a.noise_weight);
  } else {
    const int depth = t.leaf[b * 4 + 0], done = t.leaf[b * 4 + 1], winner = t.leaf[b * 4 + 2],
              player = t.leaf[b * 4 + 3];
    const int node = path[depth];
    double lv;
    if (!done) {
      const int cell = l < kAzCells ? t.leaf_board[(size_t)b * kAzCells + l] : -1;
      az_expand(t, nb, b, node, t.nnodes[b], l, gbase, cell, pr, false, 0.0);
      lv = (double)a.values[(size_t)b * a.vstride];
    } else {
      lv = winner == -1 ? 0.0 : (player == winner ? 1.0 : -1.0);
    }
    // node->update_recursive(-leaf_value): + v at the leaf, - v at its parent, ...
    const float v = (float)(-lv);
    if (l <= depth) {
      const size_t n = nb + path[depth - l];
      t.visit[n] += 1;
      t.vsum[n] += (l & 1) ? -v : v;
    }
  }
  if (a.sim + 1 >= t.S) return;
  __threadfence_block();  // the descent reads what this group just wrote

  // ---- _simulate: descend by the maximal pUCT child while the node has children
  int cell = l < kAzCells ? t.root_board[(size_t)b * kAzCells + l] : 0;
  int player = t.root_player[b];
  int node = 0, d = 0;
  if (l == 0) path[0] = 0;
  for (; d < kAzPath - 1;) {  // a board fills after 9 moves: bounded descent
    const int f = t.first[nb + node];
    if (f < 0) break;
    const int n = t.nch[nb + node];
    const int pv = t.visit[nb + node];
    double s = -__builtin_inf();
    if (l < n) {
      const size_t c = nb + f + l;
      const int cv = t.visit[c];
      const float val = cv == 0 ? 0.0f : t.vsum[c] / (float)cv;
      double pb = t.lut_pb[pv];
      pb *= t.lut_sqrt[pv] / (double)(cv + 1);
      s = pb * (double)t.prior[c] + (double)val;
    }
    int bi = l;
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) {
      const double os = __shfl_xor(s, m, kAzGroup);
      const int oi = __shfl_xor(bi, m, kAzGroup);
      if (os > s || (os == s && oi < bi)) {
        s = os;
        bi = oi;
      }
    }
    node = f + bi;
    const int mv = t.act[nb + node];
    if (l == mv) cell = player;
    player = 3 - player;
    ++d;
    if (l == 0) path[d] = node;
  }
  int bd[kAzCells];
#pragma unroll
  for (int k = 0; k < kAzCells; ++k) bd[k] = __shfl(cell, k, kAzGroup);
  int done, winner;
  az_done_winner(bd, done, winner);
  if (l == 0) {
    t.leaf[b * 4 + 0] = d;
    t.leaf[b * 4 + 1] = done;
    t.leaf[b * 4 + 2] = winner;
    t.leaf[b * 4 + 3] = player;
  }
  if (l < kAzCells) t.leaf_board[(size_t)b * kAzCells + l] = cell;
  az_write_state(a.state + (size_t)b * 27, l, cell, player);
}

// get_next_action's tail for one board: visit_count_to_action_distribution (v / T, summed in action
// order, divided), then argmax (first maximum) or a draw from the distribution (Philox keyed by seed,
// *counter and the board; the reference draws with std::random_device, so no stream is reproducible
// there)
__device__ inline void az_finalize(int b, const int *v, double temperature, int sample, uint32_t seed,
                                   const int64_t *counter, int32_t *visits_out, double *probs_out,
                                   int32_t *action_out) {
  double x[kAzCells], sum = 0.0;
  for (int k = 0; k < kAzCells; ++k) {
    x[k] = (double)v[k] / temperature;
    sum += x[k];
  }
  int best = 0;
  for (int k = 0; k < kAzCells; ++k) {
    x[k] = x[k] / sum;
    if (x[k] > x[best]) best = k;
    visits_out[(size_t)b * kAzCells + k] = v[k];
    probs_out[(size_t)b * kAzCells + k] = x[k];
  }
  if (sample) {
    const uint64_t step = counter ? (uint64_t)*counter : 0;
    const uint4 r = philox4x32_10(make_uint4((uint32_t)b, (uint32_t)step, (uint32_t)(step >> 32), 0x415au),
                                  make_uint2(seed, 0x414c5048u));
    const double u = ((double)(((uint64_t)(r.x >> 5) << 26) | (r.y >> 6)) + 0.5) * (1.0 / 9007199254740992.0);
    double cum = 0.0;
    best = -1;
    for (int k = 0; k < kAzCells; ++k) {
      cum += x[k];
      if (best < 0 && x[k] > 0.0 && u < cum) best = k;
    }
    if (best < 0)
      for (int k = kAzCells - 1; k >= 0 && best < 0; --k)
        if (x[k] > 0.0) best = k;
  }
  action_out[b] = best;
}

__global__ void az_finish_kernel(AzTree t, double temperature, int sample, uint32_t seed, const int64_t *counter,
                                 int32_t *visits_out, double *probs_out, int32_t *action_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.B) return;
  const size_t nb = (size_t)b * t.cap;
  int v[kAzCells];
  for (int k = 0; k < kAzCells; ++k) v[k] = 0;
  const int f = t.first[nb], n = t.nch[nb];
  for (int j = 0; f >= 0 && j < n; ++j) v[t.act[nb + f + j]] = t.visit[nb + f + j];
  az_finalize(b, v, temperature, sample, seed, counter, visits_out, probs_out, action_out);
}

}  // namespace lzm
