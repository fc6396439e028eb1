// Fused softmax cross-entropy forward + backward (one pass over the logits
// for max/sum, one for the gradient), plus argmax-accuracy for evaluation.
// Replaces the reference's log_softmax -> nll_loss -> nll_loss_backward ->
// log_softmax_backward chain with one kernel.
//
// logits: [B][ld] (fp32 or bf16), only the first V columns are classes
// (GPT-2 pads its vocab to a multiple of 64).  Per row: loss_i = lse - z_y.
// dlogits (optional) = (softmax - onehot) * grad_scale, written in the
// dtype requested (bf16 feeds the dgrad/wgrad GEMMs directly).
#include <algorithm>
#include <type_traits>

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
  // z_y read up front (before any thread can overwrite it when dlogits aliases logits)
  __shared__ float s_zy;
  if (threadIdx.x == 0) s_zy = (label >= 0 && label < V) ? ldv<TIn>(z, label) : 0.f;
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
  const float zy = s_zy;  // published by the barriers inside block_sum
  const float li = ignored ? 0.f : lse - zy;
  if (threadIdx.x == 0) {
    if (loss_rows) loss_rows[row] = li;                 // summed in row order by ce_sum_kernel
    else if (loss_sum) atomicAdd(loss_sum, li);
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

// Vectorised row-in-registers variant (ld % 8 == 0, ld <= NT*8*MAXC): each
// thread loads its 16-B chunks ONCE into registers, so the row is read from
// HBM once and the gradient written once (the scalar kernel above reads it
// three times).  dlogits may alias logits: every thread only rewrites the
// chunks it alone read, and z_y is taken from registers, not re-read.
template <typename TIn>
DPE_DEVICE void ce_load8(const TIn* p, float* f);
template <>
DPE_DEVICE void ce_load8<uint16_t>(const uint16_t* p, float* f) { unpack8(*(const u32x4*)p, f); }
template <>
DPE_DEVICE void ce_load8<float>(const float* p, float* f) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}

// The row is held as loaded (bf16: one u32x4 per 8 columns, half the VGPRs of fp32) and unpacked
// per pass: at ~60 VGPRs two 1024-thread blocks share a CU, so one row's block reductions overlap
// the other's loads (the LM-head rows, 50 K columns, were VGPR/occupancy-bound at one block per CU).
template <typename TIn>
struct RowChunk;
template <>
struct RowChunk<uint16_t> {
  u32x4 v;
  DPE_DEVICE void load(const uint16_t* p) { v = *(const u32x4*)p; }
  DPE_DEVICE void get(float* f) const { unpack8(v, f); }
};
template <>
struct RowChunk<float> {
  f32x4 a, b;
  DPE_DEVICE void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
  DPE_DEVICE void get(float* f) const {
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
};

template <typename TIn, typename TOut, int NT, int MAXC>
__global__ __launch_bounds__(NT, NT >= 1024 ? 8 : 1) void ce_vec_kernel(const TIn* logits, const int64_t* __restrict__ labels, int V,
                                                    int64_t ld, float grad_scale, TOut* dlogits,
                                                    float* __restrict__ loss_rows, float* __restrict__ loss_sum,
                                                    float* __restrict__ correct, int ignore_index) {
  constexpr int NW = NT / 64;
  constexpr float L2E = 1.4426950408889634f;
  __shared__ float shm[NW], shs[NW], shz[NW];
  __shared__ int sha[NW];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const TIn* z = logits + (int64_t)row * ld;
  const int nch = (int)(ld >> 3);
  const int64_t label = labels[row];
  const bool ignored = (label == ignore_index);
  const int lch = (int)(label >> 3);
  RowChunk<TIn> rc[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = tid + c * NT;
    if (ch < nch) rc[c].load(z + (int64_t)ch * 8);
  }
  // columns >= V (padding) read as -inf; only the tail chunk needs the compares
  auto chunk = [&](int c, int ch, float* f) {
    rc[c].get(f);
    if (ch * 8 + 8 > V) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (ch * 8 + e >= V) f[e] = -INFINITY;
    }
  };
  float m = -INFINITY, zy = 0.f;
  int am = 0x7fffffff;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = tid + c * NT;
    if (ch < nch) {
      float f[8];
      chunk(c, ch, f);
      if (ch == lch) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e == (int)(label & 7)) zy = f[e];
      }
      float cm = f[0];
      int ce = 0;
#pragma unroll
      for (int e = 1; e < 8; ++e)
        if (f[e] > cm) { cm = f[e]; ce = e; }
      if (cm > m) { m = cm; am = ch * 8 + ce; }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  if (lane == 0) { shm[wid] = m; sha[wid] = am; }
  __syncthreads();
  m = shm[0];
  am = sha[0];
#pragma unroll
  for (int w = 1; w < NW; ++w)
    if (shm[w] > m || (shm[w] == m && sha[w] < am)) { m = shm[w]; am = sha[w]; }
  // exp(v - m) as one fma + the bare v_exp_f32 (arguments <= 0: results in (0, 1], denormals flush)
  const float mb = -m * L2E;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = tid + c * NT;
    if (ch < nch) {
      float f[8];
      chunk(c, ch, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += __builtin_amdgcn_exp2f(fmaf(f[e], L2E, mb));
    }
  }
  s = warp_sum(s);
  zy = warp_sum(zy);
  if (lane == 0) { shs[wid] = s; shz[wid] = zy; }
  __syncthreads();
  s = 0.f;
  zy = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) { s += shs[w]; zy += shz[w]; }
  const float lse = m + __logf(s);
  const float li = ignored ? 0.f : lse - zy;
  if (tid == 0) {
    if (loss_rows) loss_rows[row] = li;                 // summed in row order by ce_sum_kernel
    else if (loss_sum) atomicAdd(loss_sum, li);
    if (correct && !ignored) atomicAdd(correct, (am == label) ? 1.f : 0.f);
  }
  if (dlogits) {
    TOut* d = dlogits + (int64_t)row * ld;
    const float k = ignored ? 0.f : grad_scale / s;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = tid + c * NT;
      if (ch < nch) {
        float f[8], g[8];
        chunk(c, ch, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = __builtin_amdgcn_exp2f(fmaf(f[e], L2E, mb)) * k;
        if (ch == lch && !ignored) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e == (int)(label & 7)) g[e] -= grad_scale;
        }
        if constexpr (sizeof(TOut) == 2) {
          *(u32x4*)(d + (int64_t)ch * 8) = pack8(g);
        } else {
          *(f32x4*)(d + (int64_t)ch * 8) = f32x4{g[0], g[1], g[2], g[3]};
          *(f32x4*)(d + (int64_t)ch * 8 + 4) = f32x4{g[4], g[5], g[6], g[7]};
        }
      }
    }
  }
}

// loss_sum[0] += sum of the B per-row losses in a fixed order (thread t takes rows t, t + 256, ...,
// then a fixed-shape tree): the reported loss is bitwise reproducible, unlike a float atomicAdd per
// row whose order follows the block schedule.  With labels: out[2] = the mean over the rows whose
// label is not ignore_index (torch's reduction="mean"; 0 valid rows -> divided by 1) and out[3] = 1 / that
// count -- the mean loss and its backward scale without the count / clamp / divide kernels of a
// torch-level reduction (the forward -> backward seam is launch-bound: ~10 tiny kernels there).
template <bool LAB>
__global__ __launch_bounds__(256) void ce_sum_kernel(const float* __restrict__ rows, int B, float* __restrict__ out,
                                                     const int64_t* __restrict__ labels, int ignore_index) {
  __shared__ float sh[256];
  __shared__ int shn[256];
  float s = 0.f;
  int n = 0;
  // 8 rows per thread per trip, all loads issued first (clamped, masked after the load): the row-serial
  // loop waited one load round trip per row (16 us for 8192 rows).  Same per-thread summation order.
  for (int i0 = threadIdx.x; i0 < B; i0 += 256 * 8) {
    float v[8];
    int64_t lb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = min(i0 + u * 256, B - 1);
      v[u] = rows[i];
      lb[u] = LAB ? labels[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (i0 + u * 256 < B) {
        s += v[u];
        n += (LAB && lb[u] != (int64_t)ignore_index) ? 1 : 0;
      }
    }
  }
  sh[threadIdx.x] = s;
  shn[threadIdx.x] = n;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sh[threadIdx.x] += sh[threadIdx.x + o];
      shn[threadIdx.x] += shn[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float tot = out[0] + sh[0];
    out[0] = tot;
    if (LAB) {
      const float cnt = (float)max(shn[0], 1);
      out[2] = tot / cnt;
      out[3] = 1.f / cnt;
    }
  }
}

// d_out = d * (*g) * (*inv_n): the mean cross-entropy's backward scale (device scalars) in one pass
template <typename T>
__global__ __launch_bounds__(256) void ce_grad_scale_kernel(const T* __restrict__ d, T* __restrict__ o, int64_t n,
                                                            const float* __restrict__ g, const float* __restrict__ inv_n) {
  const float sc = g[0] * inv_n[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if constexpr (std::is_same<T, float>::value) o[i] = d[i] * sc;
    else o[i] = f2bf(bf2f(d[i]) * sc);
  }
}

template <typename TIn, typename TOut>
bool ce_vec_launch(const TIn* logits, const int64_t* labels, int B, int V, int64_t ld, float gs, TOut* d, float* lr,
                   float* ls, float* cor, int ign, hipStream_t st) {
  if (ld % 8) return false;
  const int64_t nch = ld / 8;

#define DPE_CE_VEC(NT, MC)                                                                                         \
  if (nch <= (int64_t)(NT) * (MC)) {                                                                               \
    hipLaunchKernelGGL((ce_vec_kernel<TIn, TOut, NT, MC>), dim3(B), dim3(NT), 0, st, logits, labels, V, ld, gs, d, lr, \
                       ls, cor, ign);                                                                              \
    return true;                                                                                                   \
  }
  DPE_CE_VEC(64, 1)
  DPE_CE_VEC(128, 1)
  DPE_CE_VEC(256, 1)
  DPE_CE_VEC(256, 2)
  DPE_CE_VEC(1024, 1)
  DPE_CE_VEC(1024, 2)
  DPE_CE_VEC(1024, 4)
  DPE_CE_VEC(1024, 8)
#undef DPE_CE_VEC
  return false;
}

}  // namespace dpe

using namespace dpe;

static int dpe_cross_entropy_rows(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                                  float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* loss_sum,
                                  float* correct, int ignore_index, hipStream_t st);

// in_bf16 / out_bf16 select dtypes; dlogits may be null (eval)
extern "C" int dpe_cross_entropy(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                                 float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* loss_sum,
                                 float* correct, int ignore_index, hipStream_t st) {
  if (dlogits == logits && in_bf16 != out_bf16) return -2;  // in-place needs equal dtypes
  const int rc = dpe_cross_entropy_rows(logits, in_bf16, labels, B, V, ld, grad_scale, dlogits, out_bf16, loss_rows, loss_sum,
                                        correct, ignore_index, st);
  if (rc == 0 && loss_rows && loss_sum)
    hipLaunchKernelGGL(ce_sum_kernel<false>, dim3(1), dim3(256), 0, st, loss_rows, B, loss_sum, (const int64_t*)nullptr, 0);
  return rc;
}

// as dpe_cross_entropy, and out4[2] = mean over the non-ignored rows, out4[3] = 1 / their count (out4 = loss_sum)
extern "C" int dpe_cross_entropy_mean(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                                      float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* out4,
                                      int ignore_index, hipStream_t st) {
  if (dlogits == logits && in_bf16 != out_bf16) return -2;
  const int rc = dpe_cross_entropy_rows(logits, in_bf16, labels, B, V, ld, grad_scale, dlogits, out_bf16, loss_rows, out4,
                                        out4 + 1, ignore_index, st);
  if (rc == 0) hipLaunchKernelGGL(ce_sum_kernel<true>, dim3(1), dim3(256), 0, st, loss_rows, B, out4, labels, ignore_index);
  return rc;
}

extern "C" int dpe_ce_grad_scale(const void* d, void* o, int64_t n, int bf16, const float* g, const float* inv_n,
                                 hipStream_t st) {
  const int grid = (int)std::min<int64_t>(2048, (n + 255) / 256);
  if (grid <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(ce_grad_scale_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, (const uint16_t*)d, (uint16_t*)o, n, g,
                       inv_n);
  else
    hipLaunchKernelGGL(ce_grad_scale_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)d, (float*)o, n, g, inv_n);
  return 0;
}

static int dpe_cross_entropy_rows(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                                  float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* loss_sum,
                                  float* correct, int ignore_index, hipStream_t st) {
  if (in_bf16 ? (out_bf16 ? ce_vec_launch((const uint16_t*)logits, labels, B, V, ld, grad_scale, (uint16_t*)dlogits,
                                           loss_rows, loss_sum, correct, ignore_index, st)
                           : ce_vec_launch((const uint16_t*)logits, labels, B, V, ld, grad_scale, (float*)dlogits,
                                           loss_rows, loss_sum, correct, ignore_index, st))
              : (out_bf16 ? ce_vec_launch((const float*)logits, labels, B, V, ld, grad_scale, (uint16_t*)dlogits,
                                          loss_rows, loss_sum, correct, ignore_index, st)
                          : ce_vec_launch((const float*)logits, labels, B, V, ld, grad_scale, (float*)dlogits,
                                          loss_rows, loss_sum, correct, ignore_index, st)))
    return 0;
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
