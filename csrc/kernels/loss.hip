// Fused softmax cross-entropy forward + backward (one pass over the logits
// for max/sum, one for the gradient), plus argmax-accuracy for evaluation.
// Replaces the reference's log_softmax -> nll_loss -> nll_loss_backward ->
// log_softmax_backward chain with one kernel.
//
// logits: [B][ld] (fp32 or bf16), only the first V columns are classes
// (GPT-2 pads its vocab to a multiple of 64).  Per row: loss_i = lse - z_y.
// dlogits (optional) = (softmax - onehot) * grad_scale, written in the
// dtype requested (bf16 feeds the dgrad/wgrad GEMMs directly).
#include "common.h"

namespace dpe {

template <typename TIn>
DPE_DEVICE float ldv(const TIn* p, int64_t i);
template <>
DPE_DEVICE float ldv<float>(const float* p, int64_t i) { return p[i]; }
template <>
DPE_DEVICE float ldv<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }

template <typename TIn, typename TOut>
__global__ __launch_bounds__(1024) void ce_kernel(const TIn* __restrict__ logits, const int64_t* __restrict__ labels, int B,
                                                 int V, int64_t ld, float grad_scale, TOut* __restrict__ dlogits,
                                                 float* __restrict__ loss_rows, float* __restrict__ loss_sum,
                                                 float* __restrict__ correct, int ignore_index) {
  __shared__ float sh[32];
  __shared__ int shi[32];
  const int row = blockIdx.x;
  const TIn* z = logits + (int64_t)row * ld;
  const int64_t label = labels[row];
  const bool ignored = (label == ignore_index);
  // pass 1: max + argmax
  float m = -INFINITY;
  int am = 0;
  for (int j = threadIdx.x; j < V; j += blockDim.x) {
    const float v = ldv<TIn>(z, j);
    if (v > m) { m = v; am = j; }
  }
  // wave argmax
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { sh[wid] = m; shi[wid] = am; }
  __syncthreads();
  m = sh[0];
  am = shi[0];
  for (int w = 1; w < nw; ++w) {
    if (sh[w] > m || (sh[w] == m && shi[w] < am)) { m = sh[w]; am = shi[w]; }
  }
  __syncthreads();
  // pass 2: sum exp
  float s = 0.f;
  for (int j = threadIdx.x; j < V; j += blockDim.x) s += __expf(ldv<TIn>(z, j) - m);
  s = block_sum(s, sh);
  const float lse = m + __logf(s);
  const float zy = (label >= 0 && label < V) ? ldv<TIn>(z, label) : 0.f;
  const float li = ignored ? 0.f : lse - zy;
  if (threadIdx.x == 0) {
    if (loss_rows) loss_rows[row] = li;
    if (loss_sum) atomicAdd(loss_sum, li);
    if (correct && !ignored) atomicAdd(correct, (am == label) ? 1.f : 0.f);
  }
  if (dlogits) {
    TOut* d = dlogits + (int64_t)row * ld;
    const float inv_s = 1.f / s;
    for (int j = threadIdx.x; j < (int)ld; j += blockDim.x) {
      float g = 0.f;
      if (j < V && !ignored) g = (__expf(ldv<TIn>(z, j) - m) * inv_s - (j == label ? 1.f : 0.f)) * grad_scale;
      if constexpr (sizeof(TOut) == 2) d[j] = f2bf(g);
      else d[j] = g;
    }
  }
}

}  // namespace dpe

using namespace dpe;

// in_bf16 / out_bf16 select dtypes; dlogits may be null (eval)
extern "C" int dpe_cross_entropy(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                                 float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* loss_sum,
                                 float* correct, int ignore_index, hipStream_t st) {
  const int threads = V >= 4096 ? 1024 : 256;
  if (in_bf16) {
    if (out_bf16)
      hipLaunchKernelGGL((ce_kernel<uint16_t, uint16_t>), dim3(B), dim3(threads), 0, st, (const uint16_t*)logits, labels, B, V,
                         ld, grad_scale, (uint16_t*)dlogits, loss_rows, loss_sum, correct, ignore_index);
    else
      hipLaunchKernelGGL((ce_kernel<uint16_t, float>), dim3(B), dim3(threads), 0, st, (const uint16_t*)logits, labels, B, V, ld,
                         grad_scale, (float*)dlogits, loss_rows, loss_sum, correct, ignore_index);
  } else {
    if (out_bf16)
      hipLaunchKernelGGL((ce_kernel<float, uint16_t>), dim3(B), dim3(threads), 0, st, (const float*)logits, labels, B, V, ld,
                         grad_scale, (uint16_t*)dlogits, loss_rows, loss_sum, correct, ignore_index);
    else
      hipLaunchKernelGGL((ce_kernel<float, float>), dim3(B), dim3(threads), 0, st, (const float*)logits, labels, B, V, ld,
                         grad_scale, (float*)dlogits, loss_rows, loss_sum, correct, ignore_index);
  }
  return 0;
}
