// lzm_lstm.h — the EfficientZero reward LSTM of the recurrent step around one batched gate GEMM
// (config 3, Pong EZ).
//
// Per simulation the reference (mcts_ctree.py:756-816, efficientzero_model.py:526-574) gathers the
// leaf's (h, c) LSTM state from the per-simulation state lists, runs one nn.LSTM step on the
// flattened reward planes, and after the network zeroes the new state of every root whose
// search_len % lstm_horizon_len == 0 before appending it to the lists. As PyTorch ops that is two
// gathers, a concat, the gate GEMM, nine pointwise launches and three more for the reset mask. Here:
//   ez_lstm_input_kernel  xin[b] = [r[b] | hpool[x[b]][b]]              (gather + concat)
//   gates = xin @ W^T + bias                                           (plain GEMM: rocBLAS)
//   ez_lstm_cell_kernel   i, f, g, o = gates chunks (nn.LSTM order); c1 = s(f) c0 + s(i) tanh(g);
//                         h1 = s(o) tanh(c1) with c0 = cpool[x[b]][b]; h1 / c1 out unmasked (the
//                         value-prefix head reads h1), and masked into the next state slot
//                         (zero where search_len % horizon == 0, mcts_ctree.py:810-813).
// Both are float4-vectorised grid-stride passes: HBM/L2 bound, ~3 MB per simulation at B = 256.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lzm {

__global__ __launch_bounds__(256) void ez_lstm_input_kernel(int B, int Kr, int H, const float *r, const float *hpool,
                                                            const int32_t *x, float *xin) {
  const int K4 = (Kr + H) >> 2, Kr4 = Kr >> 2, H4 = H >> 2;
  const long long n = (long long)B * K4;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(q / K4), k = (int)(q - (long long)b * K4);
    float4 v;
    if (k < Kr4)
      v = reinterpret_cast<const float4 *>(r)[(size_t)b * Kr4 + k];
    else
      v = reinterpret_cast<const float4 *>(hpool)[((size_t)max(x[b], 0) * B + b) * H4 + (k - Kr4)];
    reinterpret_cast<float4 *>(xin)[q] = v;
  }
}

__device__ inline float lstm_sigmoid(float v) { return 1.0f / (1.0f + expf(-v)); }

__global__ __launch_bounds__(256) void ez_lstm_cell_kernel(int B, int H, const float *gates, const float *cpool,
                                                           const int32_t *x, const int32_t *search_len, int horizon,
                                                           float *h1, float *c1, float *hslot, float *cslot) {
  const int H4 = H >> 2;
  const long long n = (long long)B * H4;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(q / H4), j = (int)(q - (long long)b * H4);
    const float4 *g4 = reinterpret_cast<const float4 *>(gates) + (size_t)b * 4 * H4;
    const float4 gi = g4[j], gf = g4[H4 + j], gg = g4[2 * H4 + j], go = g4[3 * H4 + j];
    const float4 c0 = reinterpret_cast<const float4 *>(cpool)[((size_t)max(x[b], 0) * B + b) * H4 + j];
    float4 c, h;
#define LZM_LSTM_LANE(m)                                                          \
  c.m = lstm_sigmoid(gf.m) * c0.m + lstm_sigmoid(gi.m) * tanhf(gg.m);             \
  h.m = lstm_sigmoid(go.m) * tanhf(c.m);
    LZM_LSTM_LANE(x)
    LZM_LSTM_LANE(y)
    LZM_LSTM_LANE(z)
    LZM_LSTM_LANE(w)
#undef LZM_LSTM_LANE
    reinterpret_cast<float4 *>(h1)[q] = h;
    reinterpret_cast<float4 *>(c1)[q] = c;
    const bool reset = horizon > 0 && (search_len[b] % horizon) == 0;
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    reinterpret_cast<float4 *>(hslot)[q] = reset ? z : h;
    reinterpret_cast<float4 *>(cslot)[q] = reset ? z : c;
  }
}

}  // namespace lzm
