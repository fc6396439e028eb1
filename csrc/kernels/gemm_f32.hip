// fp32 GEMM on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32) -- the reference
// model's own precision.  The reference trains SimpleNet in fp32
// (/root/reference/train.py:32-50,249: nn.Linear + ReLU + Dropout(0.2) + Adam);
// this kernel gives the GPU path that precision instead of bf16, with
// reference-equal math (one fp32 rounding per product, k-ordered fma chain).
//
// One kernel, three layouts through operand strides (A(m,k) = A[m*sam + k*sak],
// B(k,n) = B[k*sbk + n*sbn]):  fwd y = x w^T, dgrad dx = dy w, wgrad dw += dy^T x.
// 64x64 block tile, 4 waves (2x2, 32x32 each = 2x2 MFMA 16x16 tiles), K-step 16
// staged through LDS.  SimpleNet's GEMMs are launch-latency bound (M = 64
// rows), so the tile is sized for few blocks, not for peak rate.
//
// Fused epilogues:
//   fwd   : y = dropout(relu(alpha*acc + bias))   Philox mask identical to dpe_dropout
//           (element j = m*N + n of the [M,N] output keeps iff philox(seed, offset + j/4)[j%4] >= p*2^32)
//   dgrad : dx = (dy w) * (mask_src > 0) * mask_scale   -- the backward of the PREVIOUS
//           layer's relu+dropout, read from its saved output (y > 0 <=> kept and positive)
//   wgrad : dw += alpha * acc                        (fp32 gradient bucket views)
#include "common.h"

namespace dpe {
namespace g32 {

constexpr int BM = 64, BN = 64, BK = 16, NT = 256;

struct G32Args {
  const float* A;
  const float* B;
  float* C;
  int64_t sam, sak, sbk, sbn, ldc;
  int M, N, K;
  const float* bias;
  float alpha;
  int relu;
  float drop_p;
  uint64_t seed, offset;
  const float* mask_src;  // dgrad: multiply by (mask_src[m*ldc+n] > 0) * mask_scale
  float mask_scale;
  int accumulate;
};

__global__ __launch_bounds__(NT) void gemm_f32_kernel(G32Args p) {
  __shared__ float As[BK][BM + 4];  // [k][m]
  __shared__ float Bs[BK][BN + 4];  // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < p.K; k0 += BK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A tile: 64 x 16, coalesced along whichever index is contiguous
      const int e = tid + i * NT;
      int mm, kk;
      if (p.sak == 1) { kk = e & 15; mm = e >> 4; } else { mm = e & 63; kk = e >> 6; }
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < p.M && gk < p.K) ? p.A[(int64_t)gm * p.sam + (int64_t)gk * p.sak] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // B tile: 16 x 64
      const int e = tid + i * NT;
      int nn, kk;
      if (p.sbk == 1) { kk = e & 15; nn = e >> 4; } else { nn = e & 63; kk = e >> 6; }
      const int gn = n0 + nn, gk = k0 + kk;
      Bs[kk][nn] = (gn < p.N && gk < p.K) ? p.B[(int64_t)gk * p.sbk + (int64_t)gn * p.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      // 16x16x4 f32: lane l holds A[m = l&15][k = l>>4] and B[k = l>>4][n = l&15]
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk + (lane >> 4)][wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk + (lane >> 4)][wc * 32 + j * 16 + (lane & 15)];
      // operands swapped (D^T issue): each lane ends up with 4 consecutive COLUMNS of one row
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // acc[i][j][r]: row m0 + wr*32 + i*16 + (lane&15), col n0 + wc*32 + j*16 + (lane>>4)*4 + r
  const uint32_t thr = (uint32_t)fminf(p.drop_p * 4294967296.f, 4294967295.f);
  const float dscale = p.drop_p < 1.f ? 1.f / (1.f - p.drop_p) : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wr * 32 + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 32 + j * 16 + (lane >> 4) * 4;
      if (n >= p.N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = p.alpha * acc[i][j][r];
        if (p.bias && n + r < p.N) v[r] += p.bias[n + r];
        if (p.relu) v[r] = fmaxf(v[r], 0.f);
      }
      if (p.drop_p > 0.f) {
        const int64_t jf = (int64_t)m * p.N + n;  // flat index of the [M, N] output (dpe_dropout's)
        if ((jf & 3) == 0 && n + 4 <= p.N) {
          const u32x4 rnd = philox4x32(p.seed, p.offset + (uint64_t)(jf >> 2), 0u);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = rnd[r] >= thr ? v[r] * dscale : 0.f;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const u32x4 rnd = philox4x32(p.seed, p.offset + (uint64_t)((jf + r) >> 2), 0u);
            v[r] = rnd[(jf + r) & 3] >= thr ? v[r] * dscale : 0.f;
          }
        }
      }
      float* dst = p.C + (int64_t)m * p.ldc + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (n + r >= p.N) break;
        float x = v[r];
        if (p.mask_src) x = p.mask_src[(int64_t)m * p.ldc + n + r] > 0.f ? x * p.mask_scale : 0.f;
        dst[r] = p.accumulate ? dst[r] + x : x;
      }
    }
  }
}

}  // namespace g32
}  // namespace dpe

using namespace dpe;

extern "C" int dpe_gemm_f32(const float* A, const float* B, float* C, int64_t sam, int64_t sak, int64_t sbk, int64_t sbn,
                            int64_t ldc, int M, int N, int K, const float* bias, float alpha, int relu, float drop_p,
                            uint64_t seed, uint64_t offset, const float* mask_src, float mask_scale, int accumulate,
                            hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  g32::G32Args p;
  p.A = A; p.B = B; p.C = C;
  p.sam = sam; p.sak = sak; p.sbk = sbk; p.sbn = sbn; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K;
  p.bias = bias; p.alpha = alpha; p.relu = relu; p.drop_p = drop_p; p.seed = seed; p.offset = offset;
  p.mask_src = mask_src; p.mask_scale = mask_scale; p.accumulate = accumulate;
  const dim3 grid((unsigned)((N + g32::BN - 1) / g32::BN), (unsigned)((M + g32::BM - 1) / g32::BM));
  hipLaunchKernelGGL(g32::gemm_f32_kernel, grid, dim3(g32::NT), 0, st, p);
  return 0;
}
