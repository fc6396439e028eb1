// LayerNorm over the last dim (GPT-2 D=768), one wave per row, 16-B lanes.
// fwd: x (f32 residual stream or bf16) -> y bf16 (feeds the next GEMM), mean/rstd f32.
// bwd: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*w; dw/db reduced
//      per block into partials, then summed (+=) into the fp32 grads.
//      dx is either written (x dtype) or ACCUMULATED into an f32 residual-stream grad.
#include "common.h"

#define DPE_LN_FIN_GROUP_MAX 8
namespace dpe {

template <bool XBF>
DPE_DEVICE void load8(const void* x, int64_t off, float* f) {
  if constexpr (XBF) {
    unpack8(*(const u32x4*)((const uint16_t*)x + off), f);
  } else {
    const f32x4 a = *(const f32x4*)((const float*)x + off), b = *(const f32x4*)((const float*)x + off + 4);
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
}

// The row stays in registers (MAXC chunks of 8 per lane): one HBM read of x,
// one write of y -- the previous 3-pass form re-read x for the variance and
// the normalisation and ran at ~1.2 TB/s.
template <bool XBF, int MAXC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, uint16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows,
                                                     int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int CH = D >> 3;
  const int64_t base = row * D;
  float f[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < CH) {
      load8<XBF>(x, base + c * 8, f[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += f[j][e];
    }
  }
  const float mean = warp_sum(s) / (float)D;
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < CH)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = f[j][e] - mean; v += d * d; }
  }
  const float rstd = rsqrtf(warp_sum(v) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < CH) {
      const f32x4 w0 = *(const f32x4*)(w + c * 8), w1 = *(const f32x4*)(w + c * 8 + 4);
      float o[8];
      o[0] = (f[j][0] - mean) * rstd * w0[0]; o[1] = (f[j][1] - mean) * rstd * w0[1];
      o[2] = (f[j][2] - mean) * rstd * w0[2]; o[3] = (f[j][3] - mean) * rstd * w0[3];
      o[4] = (f[j][4] - mean) * rstd * w1[0]; o[5] = (f[j][5] - mean) * rstd * w1[1];
      o[6] = (f[j][6] - mean) * rstd * w1[2]; o[7] = (f[j][7] - mean) * rstd * w1[3];
      if (b) {
        const f32x4 b0 = *(const f32x4*)(b + c * 8), b1 = *(const f32x4*)(b + c * 8 + 4);
        o[0] += b0[0]; o[1] += b0[1]; o[2] += b0[2]; o[3] += b0[3];
        o[4] += b1[0]; o[5] += b1[1]; o[6] += b1[2]; o[7] += b1[3];
      }
      *(u32x4*)(y + base + c * 8) = pack8(o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// ln_fwd_kernel with every load issued up front: the weights and bias (independent of the row) with the
// row itself, a tail lane (D / 8 not a multiple of 64) clamped onto the last chunk -- same loads, same
// stored bytes as its owner, its share of the sums masked.  One wave per row and every wave resident at
// once on the GPT-2 shape, so the generic kernel's second, dependent load round trip (w and b after the
// row reductions) was exposed whole.
template <bool XBF, int MAXC, bool BIAS>
__global__ __launch_bounds__(256) void ln_fwd_lean_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, uint16_t* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int64_t rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (row >= rows) return;  // (wave-uniform)
  const int CH = D >> 3;
  const int64_t base = row * D;
  float f[MAXC][8];
  f32x4 w0[MAXC], w1[MAXC], b0[MAXC], b1[MAXC];
  int cc[MAXC];
  float m[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    m[j] = c < CH ? 1.f : 0.f;
    cc[j] = min(c, CH - 1);
    load8<XBF>(x, base + cc[j] * 8, f[j]);
    w0[j] = *(const f32x4*)(w + cc[j] * 8);
    w1[j] = *(const f32x4*)(w + cc[j] * 8 + 4);
    if constexpr (BIAS) {
      b0[j] = *(const f32x4*)(b + cc[j] * 8);
      b1[j] = *(const f32x4*)(b + cc[j] * 8 + 4);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += f[j][e] * m[j];
  const float mean = warp_sum(s) / (float)D;
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = (f[j][e] - mean) * m[j]; v += d * d; }
  const float rstd = rsqrtf(warp_sum(v) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    float o[8];
    o[0] = (f[j][0] - mean) * rstd * w0[j][0]; o[1] = (f[j][1] - mean) * rstd * w0[j][1];
    o[2] = (f[j][2] - mean) * rstd * w0[j][2]; o[3] = (f[j][3] - mean) * rstd * w0[j][3];
    o[4] = (f[j][4] - mean) * rstd * w1[j][0]; o[5] = (f[j][5] - mean) * rstd * w1[j][1];
    o[6] = (f[j][6] - mean) * rstd * w1[j][2]; o[7] = (f[j][7] - mean) * rstd * w1[j][3];
    if constexpr (BIAS) {
      o[0] += b0[j][0]; o[1] += b0[j][1]; o[2] += b0[j][2]; o[3] += b0[j][3];
      o[4] += b1[j][0]; o[5] += b1[j][1]; o[6] += b1[j][2]; o[7] += b1[j][3];
    }
    *(u32x4*)(y + base + cc[j] * 8) = pack8(o);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// Row sums of the LN backward for D > 2048 (one wave per row, the whole row):
// rs[2 row] = sum(dy*w) / D, rs[2 row + 1] = sum(dy*w*xhat) / D.
template <bool XBF>
__global__ __launch_bounds__(256) void ln_bwd_rowsums_kernel(const uint16_t* __restrict__ dy, const void* __restrict__ x,
                                                             const float* __restrict__ w, const float* __restrict__ mean_in,
                                                             const float* __restrict__ rstd_in, float* __restrict__ rs,
                                                             int64_t rows, int D) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t row = blockIdx.x * 4ll + wid;
  if (row >= rows) return;
  const int64_t base = row * D;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float sg = 0.f, sgx = 0.f;
  for (int c = lane; c < (D >> 3); c += 64) {
    float d[8], f[8];
    unpack8(*(const u32x4*)(dy + base + c * 8), d);
    load8<XBF>(x, base + c * 8, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = d[e] * w[c * 8 + e];
      sg += g;
      sgx += g * (f[e] - mean) * rstd;
    }
  }
  sg = warp_sum(sg);
  sgx = warp_sum(sgx);
  if (lane == 0) {
    rs[2 * row] = sg / (float)D;
    rs[2 * row + 1] = sgx / (float)D;
  }
}

// Columns [col0, col0 + D) of rows of width Dtot, D <= 2048: each lane owns at most 4 chunks (32 columns)
// for the dw/db partials; dy and x of the row slice are loaded once and kept in registers for both
// passes.  rsums == nullptr (D == Dtot): the row sums come from the registers; else from
// ln_bwd_rowsums_kernel (rows wider than 2048: blockIdx.y walks the column chunks).
template <bool XBF, int NJ>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const uint16_t* __restrict__ dy, const void* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, void* __restrict__ dx, int dx_acc,
                                                     const float* __restrict__ res_in, uint16_t* __restrict__ dx_bf16,
                                                     float* __restrict__ part, int64_t rows, int D, int Dtot,
                                                     const float* __restrict__ rsums) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int CH = D >> 3;
  const int col0 = blockIdx.y * D;  // this block's column slice
  w += col0;
  part += col0;
  float pw[NJ][8], pb[NJ][8];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) { pw[j][e] = 0.f; pb[j][e] = 0.f; }
  for (int64_t row = blockIdx.x * 4ll + wid; row < rows; row += (int64_t)gridDim.x * 4) {
    const int64_t base = row * Dtot + col0;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float sg = 0.f, sgx = 0.f;
    float dd[NJ][8], xh[NJ][8];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < CH) {
        float f[8];
        unpack8(*(const u32x4*)(dy + base + c * 8), dd[j]);
        load8<XBF>(x, base + c * 8, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[j][e] = (f[e] - mean) * rstd;
          const float g = dd[j][e] * w[c * 8 + e];
          sg += g;
          sgx += g * xh[j][e];
          pw[j][e] += dd[j][e] * xh[j][e];
          pb[j][e] += dd[j][e];
        }
      }
    }
    if (rsums) {
      sg = rsums[2 * row];
      sgx = rsums[2 * row + 1];
    } else {
      sg = warp_sum(sg) / (float)D;
      sgx = warp_sum(sgx) / (float)D;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < CH) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rstd * (dd[j][e] * w[c * 8 + e] - sg - xh[j][e] * sgx);
        if (dx_acc) {  // fp32 residual-stream grad: dx = (res_in or dx) + dLN, optional bf16 copy
          float* p = (float*)dx + base + c * 8;
          const float* q = res_in ? res_in + base + c * 8 : p;
          f32x4 a = *(const f32x4*)q, bb = *(const f32x4*)(q + 4);
          a[0] += o[0]; a[1] += o[1]; a[2] += o[2]; a[3] += o[3];
          bb[0] += o[4]; bb[1] += o[5]; bb[2] += o[6]; bb[3] += o[7];
          *(f32x4*)p = a;
          *(f32x4*)(p + 4) = bb;
          if (dx_bf16) {
            const float t[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
            *(u32x4*)(dx_bf16 + base + c * 8) = pack8(t);
          }
        } else if (XBF) {
          *(u32x4*)((uint16_t*)dx + base + c * 8) = pack8(o);
        } else {
          float* p = (float*)dx + base + c * 8;
          *(f32x4*)p = f32x4{o[0], o[1], o[2], o[3]};
          *(f32x4*)(p + 4) = f32x4{o[4], o[5], o[6], o[7]};
        }
      }
    }
  }
  // block-reduce partials over 4 waves
  // (dynamic LDS sized [2][4][D]: 24 KiB at D = 768 instead of a fixed 64 KiB -> 6 blocks per CU)
  extern __shared__ float red_dyn[];
  float* red0 = red_dyn;          // [4][D]
  float* red1 = red_dyn + 4 * D;  // [4][D]
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < CH)
#pragma unroll
      for (int e = 0; e < 8; ++e) { red0[wid * D + c * 8 + e] = pw[j][e]; red1[wid * D + c * 8 + e] = pb[j][e]; }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += 256) {
    part[(int64_t)blockIdx.x * 2 * Dtot + i] = red0[i] + red0[D + i] + red0[2 * D + i] + red0[3 * D + i];
    part[(int64_t)blockIdx.x * 2 * Dtot + Dtot + i] = red1[i] + red1[D + i] + red1[2 * D + i] + red1[3 * D + i];
  }
}

// ln_bwd_kernel for whole rows (D <= 2048) with the output form compile-time (ACC: dx = res_in-or-dx + dLN
// in fp32; RES: res_in given; DXB: bf16 copy) and every load / store unconditional: a lane past the row's
// last chunk (D / 8 not a multiple of 64: 96 chunks at D = 768) works on the last chunk instead -- it loads
// the same operands and stores the same bytes as the lane that owns it -- and only its contribution to the
// row sums and the dw / db partials is masked.  The generic kernel's per-lane `c < CH` tests and run-time
// output forms put 7 full vmcnt waits in the row loop.
template <bool XBF, int NJ, bool ACC, bool RES, bool DXB>
__global__ __launch_bounds__(256) void ln_bwd_lean_kernel(const uint16_t* __restrict__ dy, const void* __restrict__ x,
                                                          const float* __restrict__ w, const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, void* __restrict__ dx,
                                                          const float* __restrict__ res_in, uint16_t* __restrict__ dx_bf16,
                                                          float* __restrict__ part, int64_t rows, int D) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int CH = D >> 3;
  int cc[NJ];
  bool ok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    ok[j] = c < CH;
    cc[j] = min(c, CH - 1);
  }
  float pw[NJ][8], pb[NJ][8], wv[NJ][8];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const f32x4 a = *(const f32x4*)(w + cc[j] * 8), b = *(const f32x4*)(w + cc[j] * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { wv[j][e] = a[e]; wv[j][e + 4] = b[e]; }
#pragma unroll
    for (int e = 0; e < 8; ++e) { pw[j][e] = 0.f; pb[j][e] = 0.f; }
  }
  float* __restrict__ dxf = (float*)dx;
  for (int64_t row = blockIdx.x * 4ll + wid; row < rows; row += (int64_t)gridDim.x * 4) {
    const int64_t base = row * D;
    // every operand of the row slice first (dy, x and -- independent of the row sums -- the residual-stream
    // input), then the arithmetic: one load round trip per row
    u32x4 dr[NJ], xb[NJ];
    f32x4 xr[NJ][2], rr[NJ][2];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      dr[j] = *(const u32x4*)(dy + base + cc[j] * 8);
      if constexpr (XBF) {
        xb[j] = *(const u32x4*)((const uint16_t*)x + base + cc[j] * 8);
      } else {
        xr[j][0] = *(const f32x4*)((const float*)x + base + cc[j] * 8);
        xr[j][1] = *(const f32x4*)((const float*)x + base + cc[j] * 8 + 4);
      }
      if constexpr (ACC) {
        const float* q = RES ? res_in + base + cc[j] * 8 : dxf + base + cc[j] * 8;
        rr[j][0] = *(const f32x4*)q;
        rr[j][1] = *(const f32x4*)(q + 4);
      }
    }
    const float mean = mean_in[row], rstd = rstd_in[row];
    __builtin_amdgcn_sched_barrier(0);  // (keeps the scheduler from sinking the loads to their uses)
    float sg = 0.f, sgx = 0.f;
    float dd[NJ][8], xh[NJ][8];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float f[8];
      unpack8(dr[j], dd[j]);
      if constexpr (XBF) {
        unpack8(xb[j], f);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { f[e] = xr[j][0][e]; f[e + 4] = xr[j][1][e]; }
      }
      const float m = ok[j] ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[j][e] = (f[e] - mean) * rstd;
        const float dm = dd[j][e] * m;
        const float g = dm * wv[j][e];
        sg += g;
        sgx += g * xh[j][e];
        pw[j][e] += dm * xh[j][e];
        pb[j][e] += dm;
      }
    }
    sg = warp_sum(sg) / (float)D;
    sgx = warp_sum(sgx) / (float)D;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rstd * (dd[j][e] * wv[j][e] - sg - xh[j][e] * sgx);
      if constexpr (ACC) {
        float* pp = dxf + base + cc[j] * 8;
        f32x4 a = rr[j][0], bb = rr[j][1];
        a[0] += o[0]; a[1] += o[1]; a[2] += o[2]; a[3] += o[3];
        bb[0] += o[4]; bb[1] += o[5]; bb[2] += o[6]; bb[3] += o[7];
        *(f32x4*)pp = a;
        *(f32x4*)(pp + 4) = bb;
        if constexpr (DXB) {
          const float t[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
          *(u32x4*)(dx_bf16 + base + cc[j] * 8) = pack8(t);
        }
      } else if constexpr (XBF) {
        *(u32x4*)((uint16_t*)dx + base + cc[j] * 8) = pack8(o);
      } else {
        float* pp = dxf + base + cc[j] * 8;
        *(f32x4*)pp = f32x4{o[0], o[1], o[2], o[3]};
        *(f32x4*)(pp + 4) = f32x4{o[4], o[5], o[6], o[7]};
      }
    }
  }
  extern __shared__ float red_dyn[];
  float* red0 = red_dyn;          // [4][D]
  float* red1 = red_dyn + 4 * D;  // [4][D]
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (ok[j])
#pragma unroll
      for (int e = 0; e < 8; ++e) { red0[wid * D + cc[j] * 8 + e] = pw[j][e]; red1[wid * D + cc[j] * 8 + e] = pb[j][e]; }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += 256) {
    part[(int64_t)blockIdx.x * 2 * D + i] = red0[i] + red0[D + i] + red0[2 * D + i] + red0[3 * D + i];
    part[(int64_t)blockIdx.x * 2 * D + D + i] = red1[i] + red1[D + i] + red1[2 * D + i] + red1[3 * D + i];
  }
}

// Column-parallel reduction of the [nb][2][D] partials: block = 16 columns x 64 row stripes
// (16 waves, each lane one (column, stripe); 64-B row segments), 4 independent accumulators per
// lane, fixed-order tree over the stripes; blockIdx.y picks dw (0) or db (1).  96 blocks at D = 768
// (64 columns per block gave 24 blocks on 24 CUs: ~8 us, latency-bound, 25 calls per GPT-2 step).
constexpr int LNF_W = 16, LNF_C = 16, LNF_S = LNF_W * (64 / LNF_C);
DPE_DEVICE void ln_fin_body(const float* __restrict__ part, int nb, int D, float* __restrict__ dw, float* __restrict__ db,
                            int which, int bx) {
  __shared__ float red[LNF_S][LNF_C];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cl = lane % LNF_C, stripe = wid * (64 / LNF_C) + lane / LNF_C;
  const int col = bx * LNF_C + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < D) {
    const float* src = part + (int64_t)which * D + col;
    int k = stripe;
    for (; k + 3 * LNF_S < nb; k += 4 * LNF_S) {
      a0 += src[(int64_t)k * 2 * D];
      a1 += src[(int64_t)(k + LNF_S) * 2 * D];
      a2 += src[(int64_t)(k + 2 * LNF_S) * 2 * D];
      a3 += src[(int64_t)(k + 3 * LNF_S) * 2 * D];
    }
    for (; k < nb; k += LNF_S) a0 += src[(int64_t)k * 2 * D];
  }
  red[stripe][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (threadIdx.x < LNF_C && col < D) {
    float t = 0.f;
#pragma unroll 8
    for (int w = 0; w < LNF_S; ++w) t += red[w][cl];
    if (which == 0) dw[col] += t;
    else if (db) db[col] += t;
  }
}
__global__ __launch_bounds__(64 * LNF_W) void ln_bwd_finalize_kernel(const float* __restrict__ part, int nb, int D,
                                                                     float* __restrict__ dw, float* __restrict__ db) {
  ln_fin_body(part, nb, D, dw, db, blockIdx.y, blockIdx.x);
}
// Several LayerNorms' deferred finalizes in one launch (blockIdx.z = problem): GPT-2 runs two per block,
// each a ~5 us latency-bound launch alone.
struct LnFinGroup {
  const float* part[DPE_LN_FIN_GROUP_MAX];
  float* dw[DPE_LN_FIN_GROUP_MAX];
  float* db[DPE_LN_FIN_GROUP_MAX];
  int nb[DPE_LN_FIN_GROUP_MAX], D[DPE_LN_FIN_GROUP_MAX];
};
__global__ __launch_bounds__(64 * LNF_W) void ln_bwd_finalize_group_kernel(LnFinGroup g) {
  const int z = blockIdx.z;
  if ((int)blockIdx.x * LNF_C >= g.D[z] || (blockIdx.y == 1 && !g.db[z])) return;  // (block-uniform)
  ln_fin_body(g.part[z], g.nb[z], g.D[z], g.dw[z], g.db[z], blockIdx.y, blockIdx.x);
}

}  // namespace dpe

using namespace dpe;

extern "C" int dpe_layernorm_fwd(const void* x, int x_bf16, const float* w, const float* b, uint16_t* y, float* mean,
                                 float* rstd, int64_t rows, int D, float eps, hipStream_t st) {
  if (D % 8) return -1;
  const dim3 grid((unsigned)((rows + 3) / 4));
  const int chunks = (D / 8 + 63) / 64;
  static const bool lean = [] { const char* e = getenv("DPE_LN_FWD_LEAN"); return !(e && e[0] == '0'); }();
  if (lean && chunks == 2) {  // (the GPT-2 width, 768)
#define DPE_LFL(XB, B_)                                                                                                 \
  if ((bool)x_bf16 == XB && (b != nullptr) == B_) {                                                                     \
    hipLaunchKernelGGL((ln_fwd_lean_kernel<XB, 2, B_>), grid, dim3(256), 0, st, x, w, b, y, mean, rstd, rows, D, eps);  \
    return 0;                                                                                                           \
  }
    DPE_LFL(false, true) DPE_LFL(false, false) DPE_LFL(true, true) DPE_LFL(true, false)
#undef DPE_LFL
  }
#define LNF(MC)                                                                                                        \
  if (chunks <= MC) {                                                                                                \
    if (x_bf16) hipLaunchKernelGGL((ln_fwd_kernel<true, MC>), grid, dim3(256), 0, st, x, w, b, y, mean, rstd, rows, D, eps); \
    else hipLaunchKernelGGL((ln_fwd_kernel<false, MC>), grid, dim3(256), 0, st, x, w, b, y, mean, rstd, rows, D, eps);      \
    return 0;                                                                                                        \
  }
  LNF(1)
  LNF(2)
  LNF(4)
  LNF(8)
  LNF(16)
#undef LNF
  return -1;
}

// Partial-sum blocks of the LN backward: ~2 rows per wave (4 waves per block) up to
// 1024 blocks -- 16 waves per CU on the GPT-2 shape (8192 rows); with 8 rows per
// wave (256 blocks) the row-serial wave ran latency-bound at ~2.7 TB/s.
// (Under the CU budget two rounds of half-size blocks were tried: x1.29 -> x1.24 next to 16 VALU-bound
// RCCL-sized workgroups, but twice the partials cost the finalize more than that, profiles/cu_hog_probe_r4.txt.)
extern "C" int dpe_layernorm_bwd_nblocks(int64_t rows) {
  const int64_t nb = (rows + 7) / 8;
  return (int)(nb < 1 ? 1 : (nb > 1024 ? 1024 : nb));
}

// Floats of the `part` scratch of dpe_layernorm_bwd: [nblocks][2][D] partials (+ [rows][2] row sums
// when D > 2048).
extern "C" int64_t dpe_layernorm_bwd_scratch(int64_t rows, int D) {
  return (int64_t)dpe_layernorm_bwd_nblocks(rows) * 2 * D + (D > 2048 ? 2 * rows : 0);
}

extern "C" int dpe_layernorm_bwd(const uint16_t* dy, const void* x, int x_bf16, const float* w, const float* mean,
                                 const float* rstd, void* dx, int dx_acc, const float* res_in, uint16_t* dx_bf16, float* dw,
                                 float* db, float* part, int64_t rows, int D, hipStream_t st) {
  if (D % 8) return -1;
  const int nbc = dpe_layernorm_bwd_nblocks(rows);
  // rows wider than 2048: full-row sums first, then equal column slices of <= 2048 (blockIdx.y)
  int nch = (D + 2047) / 2048;
  while (D % nch || (D / nch) % 8) ++nch;  // terminates: nch = D / 8 always divides
  const int Dc = D / nch;
  float* rs = nullptr;
  if (D > 2048) {
    rs = part + (int64_t)nbc * 2 * D;
    if (x_bf16) hipLaunchKernelGGL(ln_bwd_rowsums_kernel<true>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, dy, x, w,
                                   mean, rstd, rs, rows, D);
    else hipLaunchKernelGGL(ln_bwd_rowsums_kernel<false>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, dy, x, w, mean,
                            rstd, rs, rows, D);
  }
  const int nj = (Dc / 8 + 63) / 64;  // 16-B chunks per lane per row slice
  const size_t lds = (size_t)2 * 4 * Dc * sizeof(float);
#define DPE_LNB(XB, NJ_) \
  hipLaunchKernelGGL((ln_bwd_kernel<XB, NJ_>), dim3(nbc, nch), dim3(256), lds, st, dy, x, w, mean, rstd, dx, dx_acc, \
                     res_in, dx_bf16, part, rows, Dc, D, rs)
#define DPE_LNB_J(XB) \
  if (nj == 1) DPE_LNB(XB, 1); else if (nj == 2) DPE_LNB(XB, 2); else if (nj == 3) DPE_LNB(XB, 3); else DPE_LNB(XB, 4)
  static const bool lean = [] { const char* e = getenv("DPE_LN_BWD_LEAN"); return !(e && e[0] == '0'); }();
  bool done = false;
  if (lean && nch == 1 && !rs && nj == 2 && (dx_acc || !dx_bf16)) {
    // (the GPT-2 widths: 768 = 96 chunks; the fp32 residual-stream form first)
#define DPE_LNL(XB, A_, R_, B_)                                                                                    \
  if (!done && (bool)x_bf16 == XB && (dx_acc != 0) == A_ && (res_in != nullptr) == R_ && (dx_bf16 != nullptr) == B_) { \
    hipLaunchKernelGGL((ln_bwd_lean_kernel<XB, 2, A_, R_, B_>), dim3(nbc), dim3(256), lds, st, dy, x, w, mean, rstd, dx,  \
                       res_in, dx_bf16, part, rows, D);                                                             \
    done = true;                                                                                                   \
  }
    DPE_LNL(false, true, false, false) DPE_LNL(false, true, true, false) DPE_LNL(false, true, false, true)
    DPE_LNL(false, true, true, true) DPE_LNL(true, true, false, false) DPE_LNL(true, true, true, false)
    DPE_LNL(true, true, false, true) DPE_LNL(true, true, true, true)
    DPE_LNL(false, false, false, false) DPE_LNL(true, false, false, false)
#undef DPE_LNL
  }
  if (!done) {
    if (x_bf16) { DPE_LNB_J(true); } else { DPE_LNB_J(false); }
  }
#undef DPE_LNB_J
#undef DPE_LNB
  if (!dw && !db) return 0;  // deferred: the caller finalizes `part` later (dpe_layernorm_bwd_finalize_group)
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((D + LNF_C - 1) / LNF_C, db ? 2 : 1), dim3(64 * LNF_W), 0, st, part, nbc, D,
                     dw, db);
  return 0;
}

// The deferred finalizes of n <= DPE_LN_FIN_GROUP_MAX LayerNorm backwards (each: its `part` scratch, its row
// count, dw [D] and optional db [D], accumulated into) in one launch.
extern "C" int dpe_layernorm_bwd_finalize_group(const float* const* parts, const int64_t* rows, const int* Ds, float* const* dws,
                                                float* const* dbs, int n, hipStream_t st) {
  if (n < 1 || n > DPE_LN_FIN_GROUP_MAX) return -1;
  LnFinGroup g{};
  int dmax = 0, anyb = 0;
  for (int i = 0; i < n; ++i) {
    if (!parts[i] || !dws[i] || Ds[i] <= 0) return -1;
    g.part[i] = parts[i]; g.dw[i] = dws[i]; g.db[i] = dbs[i];
    g.nb[i] = dpe_layernorm_bwd_nblocks(rows[i]);
    g.D[i] = Ds[i];
    dmax = Ds[i] > dmax ? Ds[i] : dmax;
    anyb |= dbs[i] != nullptr;
  }
  hipLaunchKernelGGL(ln_bwd_finalize_group_kernel, dim3((dmax + LNF_C - 1) / LNF_C, anyb ? 2 : 1, n), dim3(64 * LNF_W), 0, st, g);
  return 0;
}
