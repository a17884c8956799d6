// lzm_traj.h — packing a collector's finished episodes on the device (the trajectory
// return of the sharded collector; lightzero_amd/trajectory.py holds the layout).
//
// A DeviceCollector records each env's episodes into E slots (episode k of env i in slot k % E);
// ep_count[i] counts the finished ones and consumed[i] the ones already returned. Returning them takes
// two launches and one 16-byte read-back:
//   episodes_scan_kernel  one workgroup: per env the new episodes and their rows (L + 1 each), exclusive
//                         prefix sums over the envs (episode and row offsets), and the totals
//                         {episodes, rows, slot overflow} the host reads to size the block;
//   episodes_pack_kernel  one workgroup per env: its episodes' index entries (env, L, first row), the
//                         frames of each episode as ONE contiguous copy (slot rows 0..L are adjacent in
//                         rec_frames [n][E][T+1][frame]), the scalar rows [action | reward | visits (A) |
//                         root value (| predicted value)] with row L zero except its reward column, which
//                         carries the episode's return (the env's eval_episode_return; 0 when the
//                         collector records none), and consumed[i] = ep_count[i].
// Env-major order, each env's episodes in finishing order — the order of the host loop it replaces.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lzm {

constexpr int kTrScanThreads = 1024;
constexpr int kTrPackThreads = 256;

__global__ void __launch_bounds__(kTrScanThreads)
    episodes_scan_kernel(int n, int E, const int32_t *ep_count, const int32_t *consumed, const int32_t *ep_len,
                         int32_t *env_ep_off, int64_t *env_row_off, int64_t *totals) {
  __shared__ int64_t s_ep[kTrScanThreads], s_row[kTrScanThreads];
  __shared__ int s_over;
  const int tid = threadIdx.x;
  const int chunk = (n + kTrScanThreads - 1) / kTrScanThreads;
  const int i0 = tid * chunk, i1 = min(n, i0 + chunk);
  if (tid == 0) s_over = 0;
  int64_t eps = 0, rows = 0;
  bool over = false;
  for (int i = i0; i < i1; ++i) {
    int nw = ep_count[i] - consumed[i];
    if (nw >= E) over = true;  // the running episode reuses slot ep_count % E: a returned slot was overwritten
    nw = nw < 0 ? 0 : (nw > E ? E : nw);
    for (int k = 0; k < nw; ++k) rows += (int64_t)ep_len[(size_t)i * E + (consumed[i] + k) % E] + 1;
    eps += nw;
  }
  s_ep[tid] = eps;
  s_row[tid] = rows;
  __syncthreads();
  if (over) atomicOr(&s_over, 1);
  // inclusive Hillis-Steele scan over the threads' sums
  for (int d = 1; d < kTrScanThreads; d <<= 1) {
    const int64_t ae = tid >= d ? s_ep[tid - d] : 0, ar = tid >= d ? s_row[tid - d] : 0;
    __syncthreads();
    s_ep[tid] += ae;
    s_row[tid] += ar;
    __syncthreads();
  }
  int64_t e = s_ep[tid] - eps, r = s_row[tid] - rows;  // exclusive offsets of this thread's first env
  for (int i = i0; i < i1; ++i) {
    env_ep_off[i] = (int32_t)e;
    env_row_off[i] = r;
    int nw = ep_count[i] - consumed[i];
    nw = nw < 0 ? 0 : (nw > E ? E : nw);
    for (int k = 0; k < nw; ++k) r += (int64_t)ep_len[(size_t)i * E + (consumed[i] + k) % E] + 1;
    e += nw;
  }
  if (tid == kTrScanThreads - 1) {
    totals[0] = s_ep[tid];
    totals[1] = s_row[tid];
  }
  __syncthreads();
  if (tid == 0) totals[2] = s_over;
}

struct PackArgs {
  int n, E, T, A, W, has_pred;
  int64_t frame_bytes;
  const int32_t *ep_count, *ep_len, *env_ep_off;
  int32_t *consumed;
  const int64_t *env_row_off;
  const uint8_t *rec_frames;   // [n][E][T+1][frame_bytes]
  const int32_t *rec_action;   // [n][E][T]
  const float *rec_reward;     // [n][E][T]
  const int32_t *rec_visits;   // [n][E][T][A]
  const float *rec_value;      // [n][E][T]
  const float *rec_pred;       // [n][E][T] (nullable)
  const float *ep_return;      // [n][E] (nullable)
  uint8_t *out_frames;         // [rows][frame_bytes]
  float *out_scalars;          // [rows][W]
  int64_t *out_index;          // [n_ep][3]
};

__global__ void __launch_bounds__(kTrPackThreads) episodes_pack_kernel(PackArgs p) {
  const int i = blockIdx.x, tid = threadIdx.x;
  const int c0 = p.consumed[i];
  int nw = p.ep_count[i] - c0;
  nw = nw < 0 ? 0 : (nw > p.E ? p.E : nw);
  int64_t row = p.env_row_off[i];
  const int ep0 = p.env_ep_off[i];
  const bool vec = (p.frame_bytes & 15) == 0;
  for (int k = 0; k < nw; ++k) {
    const size_t slot = (size_t)i * p.E + (size_t)((c0 + k) % p.E);
    const int L = p.ep_len[slot];
    if (tid == 0) {
      p.out_index[(size_t)(ep0 + k) * 3 + 0] = i;
      p.out_index[(size_t)(ep0 + k) * 3 + 1] = L;
      p.out_index[(size_t)(ep0 + k) * 3 + 2] = row;
    }
    // frames o_0 .. o_L: one contiguous block
    const int64_t nbytes = (int64_t)(L + 1) * p.frame_bytes;
    const uint8_t *src = p.rec_frames + slot * (size_t)(p.T + 1) * p.frame_bytes;
    uint8_t *dst = p.out_frames + (size_t)row * p.frame_bytes;
    if (vec) {
      const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
      uint4 *d4 = reinterpret_cast<uint4 *>(dst);
      for (int64_t q = tid; q < nbytes / 16; q += kTrPackThreads) d4[q] = s4[q];
    } else {
      for (int64_t q = tid; q < nbytes; q += kTrPackThreads) dst[q] = src[q];
    }
    // scalar rows (row L: zeros, the episode's return in the reward column)
    for (int t = tid; t <= L; t += kTrPackThreads) {
      float *o = p.out_scalars + (size_t)(row + t) * p.W;
      if (t == L) {
        for (int c = 0; c < p.W; ++c) o[c] = 0.0f;
        if (p.ep_return) o[1] = p.ep_return[slot];
        continue;
      }
      const size_t s = slot * p.T + t;
      o[0] = (float)p.rec_action[s];
      o[1] = p.rec_reward[s];
      for (int a = 0; a < p.A; ++a) o[2 + a] = (float)p.rec_visits[s * p.A + a];
      o[2 + p.A] = p.rec_value[s];
      if (p.has_pred) o[3 + p.A] = p.rec_pred[s];
    }
    row += L + 1;
  }
  __syncthreads();
  if (tid == 0) p.consumed[i] = p.ep_count[i];
}

}  // namespace lzm
