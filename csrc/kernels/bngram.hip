// BatchNorm-after-1x1-conv by Gram algebra (the ResNet bottleneck's conv3 -> BN3; SURVEY §7.4 hard
// part #3: BatchNorm bytes dominate once the GEMMs are fast).
//
// h3 = a2 W3^T is linear in a2 (the conv's input, [M][Cin], Cin = Cout / 4), so every per-channel
// reduction BN3 needs over h3's M rows is a reduction over a2 through two small matrices:
//   G = a2^T a2  [Cin][Cin],   s = colsum(a2)  [Cin]
//   forward:   sum_r h3[r,k]   = w_k . s            sum_r h3[r,k]^2 = w_k^T G w_k
//   backward:  P = dz3^T a2 (the weight-grad GEMM of dz3 -- the same cost as today's dh3^T a2)
//              sum_r dz3[r,k] h3[r,k] = w_k . P[k,:]
//              dW3 = sum_r dh3^T a2 = diag(a) P + diag(b) (W3 G) + c s^T          (dh3 = a dz3 + b h3 + c)
//              da2 = dh3 W3 = dz3 (diag(a) W3) + a2 (W3^T diag(b) W3) + c^T W3  -- one GEMM over the
//                    concatenated K = [dz3 | a2] x [diag(a) W3 ; Q]               (igemm AX_CAT)
// So BN3's statistics are known BEFORE conv3 runs (its epilogue writes relu(BN3(h3) + idn) directly:
// no h3 tensor, no bn_apply pass), and BN3's backward needs neither h3 nor a dh3 tensor (no
// bn_bwd_apply pass, no h3 re-read in the next block's data-grad epilogue).  The price is one read of
// a2 (a quarter of the block width) for G plus 2 M Cin^2 MFMA FLOPs, and Cin more K in the data grad.
//
// Kernels here: the Gram pass (partials per block + fixed-order reduction: deterministic), the forward
// coefficient kernel (BN3 scale / shift / mean / invstd + running stats, and u = W3 G for the
// backward), and the two backward coefficient kernels (BN3 parameter grads, the dW3 correction, the
// data grad's concatenated B operand and bias).
#include "common.h"

namespace dpe {
namespace gram {

constexpr int TR = 32;           // rows per tile (= the MFMA's K)
constexpr int TS = TR * 2 + 16;  // LDS bytes per channel row of the transposed tile (16 B pad: conflict-free b128 reads)

// Partial Gram matrix and column sums of x' = relu(x * coef[c] + coef[C + c]) (coef != nullptr) or x,
// over rows [blockIdx.x * rpb, +rpb): gp[block][C][C] (full, symmetric), sp[block][C].  x' is rounded
// to bf16 exactly as the on-load BN transform of the conv kernels rounds their MFMA operand, so G is
// the Gram matrix of the operand conv3 actually multiplies.
template <int C>
__global__ __launch_bounds__(256) void gram_partial_kernel(const uint16_t* __restrict__ x, const float* __restrict__ coef,
                                                           int64_t M, int rpb, float* __restrict__ gp,
                                                           float* __restrict__ sp) {
  constexpr int NB = C / 16, NF = NB * (NB + 1) / 2, FPW = (NF + 3) / 4;
  constexpr int CPR = C / 8;          // 16-B chunks per row
  constexpr int CPT = TR * CPR / 256; // chunks per thread per tile
  static_assert(CPT >= 1 && CPT * 256 == TR * CPR, "tile split");
  __shared__ __attribute__((aligned(16))) char tile[2][C * TS];
  __shared__ float red[256 / CPR * 8 + 8];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min<int64_t>(M, r0 + rpb);
  const int ntile = r0 < r1 ? (int)((r1 - r0 + TR - 1) / TR) : 0;

  // this thread's chunks: q = tid + 256 i -> row q / CPR, channels 8 (q % CPR) .. +7 (the same
  // channels on every tile: CPR divides 256)
  const int cc = tid % CPR;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = coef ? coef[8 * cc + e] : 1.f;
    sh[e] = coef ? coef[C + 8 * cc + e] : 0.f;
  }
  float csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;

  // fragments (I <= J) of wave wid: f = wid + 4 i
  int fi[FPW], fj[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    int f = wid + 4 * i, I = 0;
    if (f >= NF) f = NF - 1;  // (padding slot: recomputes a valid fragment, never stored)
    while (f >= NB - I) { f -= NB - I; ++I; }
    fi[i] = I;
    fj[i] = I + f;
  }
  f32x4 acc[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ld[CPT];
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int q = tid + 256 * i, row = q / CPR;
      const int64_t m = r0 + (int64_t)t * TR + row;
      ld[i] = m < r1 ? *(const u32x4*)(x + m * C + 8 * cc) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  if (ntile > 0) load(0);
  for (int t = 0; t < ntile; ++t) {
    char* T = tile[t & 1];
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int q = tid + 256 * i, row = q / CPR;
      const bool valid = r0 + (int64_t)t * TR + row < r1;
      float f[8];
      unpack8(ld[i], f);
      if (coef) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = valid ? fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f) : 0.f;
      }
      const u32x4 pk = pack8(f);
      unpack8(pk, f);  // the rounded operand
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[e] += f[e];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        *(uint16_t*)(T + (8 * cc + 2 * e) * TS + row * 2) = (uint16_t)(pk[e] & 0xffffu);
        *(uint16_t*)(T + (8 * cc + 2 * e + 1) * TS + row * 2) = (uint16_t)(pk[e] >> 16);
      }
    }
    if (t + 1 < ntile) load(t + 1);  // in flight across the MFMAs below
    __syncthreads();
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, *(const u32x4*)(T + (16 * fi[i] + li) * TS + g * 16));
      const bf16x8 b = __builtin_bit_cast(bf16x8, *(const u32x4*)(T + (16 * fj[i] + li) * TS + g * 16));
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
    }
    // (the next tile writes the other buffer; this one is rewritten two tiles on, after the barrier
    // above has been passed by every wave that read it)
  }
  // partial G: lane holds D[4 (lane / 16) + e][lane % 16] of fragment (I, J); mirrored below the diagonal
  float* G = gp + (int64_t)blockIdx.x * C * C;
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    if (wid + 4 * i >= NF) continue;
    const int I = fi[i], J = fj[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 16 * I + 4 * g + e, c = 16 * J + li;
      G[(int64_t)r * C + c] = acc[i][e];
      if (I != J) G[(int64_t)c * C + r] = acc[i][e];
    }
  }
  // column sums: threads tid, tid + CPR, ... hold the same channels (fixed-order LDS reduction)
  __syncthreads();
  float* rs = (float*)tile[0];  // [256][8]
#pragma unroll
  for (int e = 0; e < 8; ++e) rs[tid * 8 + e] = csum[e];
  __syncthreads();
  if (tid < CPR) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    for (int k = tid; k < 256; k += CPR)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rs[k * 8 + e];
#pragma unroll
    for (int e = 0; e < 8; ++e) sp[(int64_t)blockIdx.x * C + 8 * tid + e] = v[e];
  }
  (void)red;
}

// G[i] = sum_b gp[b][i] (i over C*C, then the C column sums), in block order, in double
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ gp, const float* __restrict__ sp, int nb,
                                                          int C, float* __restrict__ G, float* __restrict__ s) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t cc = (int64_t)C * C;
  if (i < cc) {
    double a = 0.0;
    int b = 0;
    for (; b + 3 < nb; b += 4) {
      const float v0 = gp[(int64_t)b * cc + i], v1 = gp[(int64_t)(b + 1) * cc + i];
      const float v2 = gp[(int64_t)(b + 2) * cc + i], v3 = gp[(int64_t)(b + 3) * cc + i];
      a += v0; a += v1; a += v2; a += v3;
    }
    for (; b < nb; ++b) a += gp[(int64_t)b * cc + i];
    G[i] = (float)a;
  } else if (i < cc + C) {
    const int c = (int)(i - cc);
    double a = 0.0;
    for (int b = 0; b < nb; ++b) a += sp[(int64_t)b * C + c];
    s[c] = (float)a;
  }
}

constexpr int KPB = 8;  // output channels per block of the coefficient kernels

// Forward: per output channel k of conv3 (weights w [Cout][Cin] bf16), u[k][:] = w_k G and
//   mean = (w_k . s) / M,  E[h^2] = (w_k . u[k]) / M  ->  coef [4][Cout] = scale, shift, mean, invstd
// (the layout of bn_finalize_kernel), running stats updated as there (unbiased variance).
__global__ __launch_bounds__(256) void gram_coef_kernel(const float* __restrict__ G, const float* __restrict__ s,
                                                        const uint16_t* __restrict__ w, int Cin, int Cout, int64_t M,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        float* __restrict__ rmean, float* __restrict__ rvar, float momentum,
                                                        float eps, float* __restrict__ coef, float* __restrict__ u) {
  extern __shared__ float wl[];  // [KPB][Cin]
  __shared__ double red[2][KPB][4];
  const int k0 = blockIdx.x * KPB, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < KPB * Cin; i += 256) {
    const int kk = i / Cin, j = i - kk * Cin;
    wl[i] = k0 + kk < Cout ? bf2f(w[(int64_t)(k0 + kk) * Cin + j]) : 0.f;
  }
  __syncthreads();
  double e2[KPB], mu[KPB];
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) { e2[kk] = 0.0; mu[kk] = 0.0; }
  for (int j = tid; j < Cin; j += 256) {
    float acc[KPB];
#pragma unroll
    for (int kk = 0; kk < KPB; ++kk) acc[kk] = 0.f;
    for (int jp = 0; jp < Cin; ++jp) {
      const float gv = G[(int64_t)jp * Cin + j];
#pragma unroll
      for (int kk = 0; kk < KPB; ++kk) acc[kk] = fmaf(wl[kk * Cin + jp], gv, acc[kk]);
    }
    const float sj = s[j];
#pragma unroll
    for (int kk = 0; kk < KPB; ++kk) {
      if (k0 + kk < Cout) u[(int64_t)(k0 + kk) * Cin + j] = acc[kk];
      e2[kk] += (double)acc[kk] * wl[kk * Cin + j];
      mu[kk] += (double)wl[kk * Cin + j] * sj;
    }
  }
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) {
    for (int o = 32; o > 0; o >>= 1) {
      e2[kk] += __shfl_xor(e2[kk], o, 64);
      mu[kk] += __shfl_xor(mu[kk], o, 64);
    }
    if (lane == 0) { red[0][kk][wid] = e2[kk]; red[1][kk][wid] = mu[kk]; }
  }
  __syncthreads();
  if (tid < KPB && k0 + tid < Cout) {
    const int k = k0 + tid;
    double E2 = 0.0, S = 0.0;
    for (int q = 0; q < 4; ++q) { E2 += red[0][tid][q]; S += red[1][tid][q]; }
    const double mean = S / (double)M;
    double var = E2 / (double)M - mean * mean;
    if (var < 0) var = 0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float gm = gamma ? gamma[k] : 1.f, bt = beta ? beta[k] : 0.f;
    const float sc = gm * invstd;
    coef[k] = sc;
    coef[Cout + k] = bt - (float)mean * sc;
    coef[2 * Cout + k] = (float)mean;
    coef[3 * Cout + k] = invstd;
    if (rmean) {
      const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
      rmean[k] = (1.f - momentum) * rmean[k] + momentum * (float)mean;
      rvar[k] = (1.f - momentum) * rvar[k] + momentum * (float)unbiased;
    }
  }
}

// Backward, per output channel k.  part [2][Cout][RG]: row 0 = partial sums of dz3 (row 1 unused);
// P [Cout][Cin] = dz3^T a2; u = W3 G; s = colsum(a2); coef3 = BN3's (scale, shift, mean, invstd).
//   Sdz = sum dz,  Sdzh = w_k . P[k],  Sdzx = invstd (Sdzh - mean Sdz)
//   dgamma += Sdzx, dbeta += Sdz;  a = gamma invstd, b = -a invstd Sdzx / M, c = -a Sdz / M - b mean
//   dW3[k] += a P[k] + b u[k] + c s                       (fp32, the gradient buffer)
//   bcat[k][:] = bf16(a w_k)                              (the data grad's B rows 0 .. Cout-1)
//   abc [3][Cout] = (a, b, c) for gram_q_kernel
__global__ __launch_bounds__(256) void gram_bwd_kernel(const float* __restrict__ part, int rg, const float* __restrict__ P,
                                                       const uint16_t* __restrict__ w, const float* __restrict__ u,
                                                       const float* __restrict__ s, const float* __restrict__ coef3,
                                                       const float* __restrict__ gamma, int Cin, int Cout, int64_t M,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                       float* __restrict__ dw, uint16_t* __restrict__ bcat,
                                                       float* __restrict__ abc) {
  __shared__ double red[2][KPB][4];
  __shared__ float kc[KPB][3];
  const int k0 = blockIdx.x * KPB, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double sdz[KPB], sdzh[KPB];
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) { sdz[kk] = 0.0; sdzh[kk] = 0.0; }
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) {
    const int k = k0 + kk;
    if (k >= Cout) continue;
    for (int j = tid; j < Cin; j += 256) sdzh[kk] += (double)bf2f(w[(int64_t)k * Cin + j]) * P[(int64_t)k * Cin + j];
    for (int q = tid; q < rg; q += 256) sdz[kk] += part[(int64_t)k * rg + q];
  }
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) {
    for (int o = 32; o > 0; o >>= 1) {
      sdz[kk] += __shfl_xor(sdz[kk], o, 64);
      sdzh[kk] += __shfl_xor(sdzh[kk], o, 64);
    }
    if (lane == 0) { red[0][kk][wid] = sdz[kk]; red[1][kk][wid] = sdzh[kk]; }
  }
  __syncthreads();
  if (tid < KPB) {
    const int k = k0 + tid;
    float a = 0.f, b = 0.f, c = 0.f;
    if (k < Cout) {
      double Sdz = 0.0, Sdzh = 0.0;
      for (int q = 0; q < 4; ++q) { Sdz += red[0][tid][q]; Sdzh += red[1][tid][q]; }
      const double mean = coef3[2 * Cout + k], invstd = coef3[3 * Cout + k];
      const double Sdzx = invstd * (Sdzh - mean * Sdz);
      const double gm = gamma ? gamma[k] : 1.0;
      if (dgamma) dgamma[k] += (float)Sdzx;
      if (dbeta) dbeta[k] += (float)Sdz;
      const double A = gm * invstd;
      const double B = -A * invstd * Sdzx / (double)M;
      const double Cc = -A * Sdz / (double)M - B * mean;
      a = (float)A; b = (float)B; c = (float)Cc;
      abc[k] = a;
      abc[Cout + k] = b;
      abc[2 * Cout + k] = c;
    }
    kc[tid][0] = a; kc[tid][1] = b; kc[tid][2] = c;
  }
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < KPB; ++kk) {
    const int k = k0 + kk;
    if (k >= Cout) continue;
    const float a = kc[kk][0], b = kc[kk][1], c = kc[kk][2];
    for (int j = tid; j < Cin; j += 256) {
      const int64_t o = (int64_t)k * Cin + j;
      const float wv = bf2f(w[o]);
      dw[o] += fmaf(a, P[o], fmaf(b, u[o], c * s[j]));
      bcat[o] = f2bf(a * wv);
    }
  }
}

// Backward: the data grad's B rows Cout + j' (Q = W3^T diag(b) W3, bf16) and its bias e = c^T W3 (fp32).
// One thread per (j', j); the j' == 0 threads also produce e[j].
__global__ __launch_bounds__(256) void gram_q_kernel(const uint16_t* __restrict__ w, const float* __restrict__ abc, int Cin,
                                                     int Cout, uint16_t* __restrict__ bcat, float* __restrict__ ebias) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)Cin * Cin) return;
  const int jp = (int)(i / Cin), j = (int)(i - (int64_t)jp * Cin);
  const float* b = abc + Cout;
  const float* c = abc + 2 * Cout;
  float q = 0.f, e = 0.f;
  for (int k = 0; k < Cout; ++k) {
    const float wj = bf2f(w[(int64_t)k * Cin + j]);
    q = fmaf(bf2f(w[(int64_t)k * Cin + jp]) * b[k], wj, q);
    if (jp == 0) e = fmaf(c[k], wj, e);
  }
  bcat[(int64_t)(Cout + jp) * Cin + j] = f2bf(q);
  if (jp == 0) ebias[j] = e;
}

}  // namespace gram
}  // namespace dpe

using namespace dpe;

// Gram pass: x [M][C] bf16 (C in {64, 128, 256}), coef = BN [scale | shift] applied with ReLU on load (or
// nullptr); ws >= dpe_gram_ws_floats(M, C) floats.  Writes G [C][C], s [C].
extern "C" int dpe_gram_blocks(int64_t M, int C) {
  const int nb = C <= 128 ? 256 : 128;
  return (int)std::min<int64_t>(nb, std::max<int64_t>(1, (M + gram::TR - 1) / gram::TR));
}
extern "C" int64_t dpe_gram_ws_floats(int64_t M, int C) { return (int64_t)dpe_gram_blocks(M, C) * ((int64_t)C * C + C); }

extern "C" int dpe_gram(const uint16_t* x, const float* coef, int64_t M, int C, float* ws, float* G, float* s,
                        hipStream_t st) {
  if (C != 64 && C != 128 && C != 256) return -1;
  const int nb = dpe_gram_blocks(M, C);
  const int64_t tiles = (M + gram::TR - 1) / gram::TR;
  const int rpb = (int)(((tiles + nb - 1) / nb) * gram::TR);
  float* gp = ws;
  float* sp = ws + (int64_t)nb * C * C;
  if (C == 64) hipLaunchKernelGGL(gram::gram_partial_kernel<64>, dim3(nb), dim3(256), 0, st, x, coef, M, rpb, gp, sp);
  else if (C == 128) hipLaunchKernelGGL(gram::gram_partial_kernel<128>, dim3(nb), dim3(256), 0, st, x, coef, M, rpb, gp, sp);
  else hipLaunchKernelGGL(gram::gram_partial_kernel<256>, dim3(nb), dim3(256), 0, st, x, coef, M, rpb, gp, sp);
  const int64_t n = (int64_t)C * C + C;
  hipLaunchKernelGGL(gram::gram_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, gp, sp, nb, C, G, s);
  return 0;
}

extern "C" int dpe_gram_coef(const float* G, const float* s, const uint16_t* w, int Cin, int Cout, int64_t M,
                             const float* gamma, const float* beta, float* rmean, float* rvar, float momentum, float eps,
                             float* coef, float* u, hipStream_t st) {
  const unsigned nb = (unsigned)((Cout + gram::KPB - 1) / gram::KPB);
  hipLaunchKernelGGL(gram::gram_coef_kernel, dim3(nb), dim3(256), gram::KPB * Cin * sizeof(float), st, G, s, w, Cin, Cout,
                     M, gamma, beta, rmean, rvar, momentum, eps, coef, u);
  return 0;
}

extern "C" int dpe_gram_bwd(const float* part, int rg, const float* P, const uint16_t* w, const float* u, const float* s,
                            const float* coef3, const float* gamma, int Cin, int Cout, int64_t M, float* dgamma,
                            float* dbeta, float* dw, uint16_t* bcat, float* abc, float* ebias, hipStream_t st) {
  const unsigned nb = (unsigned)((Cout + gram::KPB - 1) / gram::KPB);
  hipLaunchKernelGGL(gram::gram_bwd_kernel, dim3(nb), dim3(256), 0, st, part, rg, P, w, u, s, coef3, gamma, Cin, Cout, M,
                     dgamma, dbeta, dw, bcat, abc);
  const int64_t n = (int64_t)Cin * Cin;
  hipLaunchKernelGGL(gram::gram_q_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, abc, Cin, Cout, bcat,
                     ebias);
  return 0;
}
