// Implicit-GEMM engine for gfx950: dense GEMM (NT / NN / TN) and NHWC
// convolution forward / data-grad / weight-grad on bf16 MFMA
// (v_mfma_f32_16x16x32_bf16), fp32 accumulate.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves in a 2x2 grid; each wave owns a (BM/2)x(BN/2)
//     sub-tile as (BM/32)x(BN/32) 16x16 MFMA tiles.
//   * BK = 32; global -> registers -> LDS staging (register staging because
//     the conv loaders gather / zero-pad), double-buffered LDS, ONE barrier
//     per K-step: next tile's global loads are issued before the MFMAs of the
//     current tile and written to the other buffer after them (T14 split).
//   * K-contiguous operands live in a [rows][32] LDS image read with
//     ds_read_b128 and XOR-swizzled so each 16-lane group of the read hits 16
//     distinct 16-B bank slots (swizzle g = {0,2,3,1} on (row>>2)&3).
//   * M/N-contiguous operands (weight-grad A = dy^T, weight-grad B = im2col x,
//     data-grad B = weights) live in a [32][cols] image read with the CDNA4
//     transposing ds_read_b64_tr_b16 (T10); chunk XOR-swizzle chosen so both
//     32-lane halves of every transposed read are conflict-free.
//   * MFMA operands are issued swapped (D^T = B^T A^T) so each lane ends up
//     holding 4 consecutive output COLUMNS of one output row: the epilogue
//     writes 8-byte packed bf16 to an LDS C tile, then stores whole 16-byte
//     row chunks (coalesced), optionally adding a residual and accumulating
//     per-column sum / sum-of-squares for a following BatchNorm.
//   * Workgroup ids are remapped XCD-aware (bijective) with N-tiles fastest
//     so the blocks that share an A row-panel share an L2.
#include "common.h"
#include "igemm.h"

namespace dpe {

constexpr int BK = 32;
constexpr int NT = 256;

// ---------------------------------------------------------------- LDS images
// K-contiguous image: row r holds 32 bf16 (64 B) as 4 chunks of 16 B.
DPE_DEVICE int kimg_off(int row, int chunk) {
  const int g = (0x78 >> (((row >> 2) & 3) << 1)) & 3;  // g = {0,2,3,1}
  return row * 64 + ((chunk ^ g) << 4);
}

// M/N-contiguous image: row k holds COLS bf16 as COLS/8 chunks of 16 B.
template <int COLS>
DPE_DEVICE int mnimg_off(int k, int chunk) {
  int h;
  if constexpr (COLS == 128) {
    h = ((k & 3) | (((k >> 3) & 1) << 2)) << 1;
  } else {
    static_assert(COLS == 64, "mn image supports 64/128 columns");
    h = (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  }
  return k * (COLS * 2) + ((chunk ^ h) << 4);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DPE_DEVICE bf16x8 kfrag(const char* img, int r0) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15);
  u32x4 v = *(const u32x4*)(img + kimg_off(row, lane >> 4));
  return __builtin_bit_cast(bf16x8, v);
}

template <int COLS>
DPE_DEVICE bf16x8 mnfrag(const char* img, int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k1 = 8 * g + q, k2 = k1 + 4;
  const int mc = (c0 >> 3) + (p >> 1);
  const int sub = (p & 1) * 8;
  const char* a1 = img + mnimg_off<COLS>(k1, mc) + sub;
  const char* a2 = img + mnimg_off<COLS>(k2, mc) + sub;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

DPE_DEVICE u32x4 ld16(const uint16_t* p) { return *(const u32x4*)p; }
DPE_DEVICE u32x4 zero16() { u32x4 z; z[0] = z[1] = z[2] = z[3] = 0u; return z; }

// Out-of-range chunks (conv padding, M/N/K tails) load from this zero page: the
// address is selected (v_cndmask), the load is unconditional -- no branch per chunk.
__device__ __attribute__((aligned(64))) uint16_t igemm_zero_page[32];
DPE_DEVICE u32x4 ld16z(bool v, const uint16_t* p) { return *(const u32x4*)(v ? p : igemm_zero_page); }

// ------------------------------------------------------------------ loaders
// K-contiguous loaders: tile [ROWS][32]; chunk c -> row c>>2, kchunk c&3.
template <int ROWS, int KIND>
struct KLoader {
  static constexpr int NC = ROWS * 4 / NT;  // chunks per thread
  const uint16_t* base[NC];
  int row[NC];
  bool vrow[NC];
  // conv state per chunk
  int ihb[NC], iwb[NC];   // fwd: oh*sh-ph, ow*sw-pw ; dgrad: h+ph, w+pw
  int ci[NC], s[NC], r[NC];
  int kk[NC];             // absolute k of the chunk

  DPE_DEVICE void init(const IgemmArgs& p, const uint16_t* ptr, int64_t ld, int rows_total, int r0, int kb) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      row[i] = c >> 2;
      const int kc = c & 3;
      const int gr = r0 + row[i];
      vrow[i] = gr < rows_total;
      kk[i] = kb + kc * 8;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        base[i] = ptr + (int64_t)(vrow[i] ? gr : 0) * ld + kk[i];
      } else {
        const ConvGeom& g = p.g;
        const int grr = vrow[i] ? gr : 0;
        if constexpr (KIND == A_CONV_FWD) {
          const int ow = grr % g.OW, t = grr / g.OW, oh = t % g.OH, n = t / g.OH;
          ihb[i] = oh * g.sh - g.ph;
          iwb[i] = ow * g.sw - g.pw;
          base[i] = ptr + (int64_t)n * g.H * g.W * g.C;
          const int kc0 = kk[i];
          ci[i] = kc0 % g.C;
          const int rs = kc0 / g.C;
          s[i] = rs % g.S;
          r[i] = rs / g.S;
        } else {  // A_CONV_DGRAD: rows over input pixels, k = (r, s, co)
          const int w = grr % g.W, t = grr / g.W, h = t % g.H, n = t / g.H;
          ihb[i] = h + g.ph;
          iwb[i] = w + g.pw;
          base[i] = ptr + (int64_t)n * g.OH * g.OW * g.K;
          const int kc0 = kk[i];
          ci[i] = kc0 % g.K;
          const int rs = kc0 / g.K;
          s[i] = rs % g.S;
          r[i] = rs / g.S;
        }
      }
    }
  }

  DPE_DEVICE void load(const IgemmArgs& p, int kend, u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      bool v = vrow[i] && kk[i] < kend;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        regs[i] = ld16z(v, base[i]);
      } else if constexpr (KIND == A_CONV_FWD) {
        const ConvGeom& g = p.g;
        const int ih = ihb[i] + r[i] * g.dh, iw = iwb[i] + s[i] * g.dw;
        v = v && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        regs[i] = ld16z(v, base[i] + ((int64_t)ih * g.W + iw) * g.C + ci[i]);
      } else {  // A_CONV_DGRAD
        const ConvGeom& g = p.g;
        const int oh_ = ihb[i] - r[i] * g.dh, ow_ = iwb[i] - s[i] * g.dw;
        const int oh = oh_ / g.sh, ow = ow_ / g.sw;
        v = v && oh_ >= 0 && ow_ >= 0 && oh * g.sh == oh_ && ow * g.sw == ow_ && oh < g.OH && ow < g.OW;
        regs[i] = ld16z(v, base[i] + ((int64_t)oh * g.OW + ow) * g.K + ci[i]);
      }
    }
  }

  DPE_DEVICE void advance(const IgemmArgs& p) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      kk[i] += BK;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        base[i] += BK;
      } else {
        const int C = (KIND == A_CONV_FWD) ? p.g.C : p.g.K;
        ci[i] += BK;
        while (ci[i] >= C) {
          ci[i] -= C;
          if (++s[i] == p.g.S) { s[i] = 0; ++r[i]; }
        }
      }
    }
  }

  DPE_DEVICE void store(char* img, const u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      *(u32x4*)(img + kimg_off(row[i], c & 3)) = regs[i];
    }
  }
};

// M/N-contiguous loaders: tile [32][COLS]; chunk c -> krow c/(COLS/8), col chunk c%(COLS/8).
template <int COLS, int KIND>
struct MNLoader {
  static constexpr int CPR = COLS / 8;
  static constexpr int NC = BK * CPR / NT;
  const uint16_t* base[NC];
  int krow[NC], cc[NC];
  bool vcol[NC];
  int kk[NC];
  // dgrad weights: k = (t,u,co) -> co, virtual taps (t,u) -> real (r,s)
  int co[NC], tt[NC], uu[NC];
  // wgrad im2col: k = pixel -> (img, oh, ow); column chunk -> (r, s, ci)
  int img[NC], oh[NC], ow[NC];
  int roff[NC], soff[NC];

  DPE_DEVICE void init(const IgemmArgs& p, const uint16_t* ptr, int64_t ld, int cols_total, int c0, int kb) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      krow[i] = c / CPR;
      cc[i] = c % CPR;
      const int gc = c0 + cc[i] * 8;
      vcol[i] = gc < cols_total;
      const int gcc = vcol[i] ? gc : 0;
      kk[i] = kb + krow[i];
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        base[i] = ptr + (int64_t)kk[i] * ld + gcc;
      } else if constexpr (KIND == B_CONV_DGRAD) {
        const ConvGeom& g = p.g;
        co[i] = kk[i] % g.K;
        const int rs = kk[i] / g.K;
        tt[i] = rs / g.S;
        uu[i] = rs % g.S;
        base[i] = ptr + gcc;  // + co*RR*SS*C + (r*SS + s)*C
      } else {  // B_CONV_WGRAD
        const ConvGeom& g = p.g;
        const int cin = gcc % g.C, t = gcc / g.C;
        const int ss = t % g.S, rr = t / g.S;
        roff[i] = rr * g.dh - g.ph;
        soff[i] = ss * g.dw - g.pw;
        base[i] = ptr + cin;
        const int px = kk[i];
        ow[i] = px % g.OW;
        const int tt = px / g.OW;
        oh[i] = tt % g.OH;
        img[i] = tt / g.OH;
      }
    }
  }

  DPE_DEVICE void load(const IgemmArgs& p, int kend, u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      bool v = vcol[i] && kk[i] < kend;
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        regs[i] = ld16z(v, base[i]);
      } else if constexpr (KIND == B_CONV_DGRAD) {
        const ConvGeom& g = p.g;
        const int r = g.pr0 + g.psh * tt[i], s_ = g.ps0 + g.psw * uu[i];
        regs[i] = ld16z(v, base[i] + (int64_t)co[i] * g.RR * g.SS * g.C + (int64_t)(r * g.SS + s_) * g.C);
      } else {
        const ConvGeom& g = p.g;
        const int ih = oh[i] * g.sh + roff[i], iw = ow[i] * g.sw + soff[i];
        v = v && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        regs[i] = ld16z(v, base[i] + (((int64_t)img[i] * g.H + ih) * g.W + iw) * g.C);
      }
    }
  }

  DPE_DEVICE void advance(const IgemmArgs& p, int64_t ld) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      kk[i] += BK;
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        base[i] += BK * ld;
      } else if constexpr (KIND == B_CONV_DGRAD) {
        co[i] += BK;
        while (co[i] >= p.g.K) {
          co[i] -= p.g.K;
          if (++uu[i] == p.g.S) { uu[i] = 0; ++tt[i]; }
        }
      } else {
        ow[i] += BK;
        while (ow[i] >= p.g.OW) {
          ow[i] -= p.g.OW;
          if (++oh[i] == p.g.OH) { oh[i] = 0; ++img[i]; }
        }
      }
    }
  }

  DPE_DEVICE void store(char* img_, const u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) *(u32x4*)(img_ + mnimg_off<COLS>(krow[i], cc[i])) = regs[i];
  }
};

template <int KIND> struct IsK { static constexpr bool v = (KIND == A_DENSE_K || KIND == A_CONV_FWD || KIND == A_CONV_DGRAD); };
template <int KIND> struct IsBK { static constexpr bool v = (KIND == B_DENSE_K); };

DPE_DEVICE float act_fn(float x, int act) {
  if (act == ACT_RELU) return fmaxf(x, 0.f);
  if (act == ACT_GELU) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (x + k1 * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  }
  return x;
}

// -------------------------------------------------------------------- kernel
template <int BM, int BN, int AL, int BL, int EPI>
__global__ __launch_bounds__(NT) void igemm_kernel(IgemmArgs p) {
  constexpr bool AK = IsK<AL>::v;
  constexpr bool BKc = IsBK<BL>::v;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CROW = BN * 2 + 16;
  constexpr int LDS_MAIN = 2 * STAGE;
  constexpr int LDS_C = (EPI == EPI_BF16 || EPI == EPI_BF16_BNB) ? (BM * CROW + 2 * 4 * BN * 4)
                        : (EPI == EPI_ATOMIC_F32 ? (BM / 2) * (BN + 4) * 4 : 0);
  constexpr int LDS = LDS_MAIN > LDS_C ? LDS_MAIN : LDS_C;
  constexpr int RM = BM / 32, RN = BN / 32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tilesM = (p.M + BM - 1) / BM;
  const int ntile = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntile, split = bid / ntile;
  const int tm = tile / tilesN, tn = tile % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = split * p.k_split;
  const int ke = min(p.K, kb + p.k_split);
  const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);

  using ALdr = typename std::conditional<AK, KLoader<BM, AL>, MNLoader<BM, AL>>::type;
  using BLdr = typename std::conditional<BKc, KLoader<BN, BL>, MNLoader<BN, BL>>::type;
  ALdr al;
  BLdr bl;
  if constexpr (AK) al.init(p, p.A, p.lda, p.M, m0, kb); else al.init(p, p.A, p.lda, p.M, m0, kb);
  if constexpr (BKc) bl.init(p, p.B, p.ldb, p.N, n0, kb); else bl.init(p, p.B, p.ldb, p.N, n0, kb);

  u32x4 ra[ALdr::NC], rb[BLdr::NC];
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int cur = 0;
  if (kb < ke) {
    al.load(p, ke, ra);
    bl.load(p, ke, rb);
    al.store(smem, ra);
    bl.store(smem + A_BYTES, rb);
    if constexpr (AK) al.advance(p); else al.advance(p, p.lda);
    if constexpr (BKc) bl.advance(p); else bl.advance(p, p.ldb);
  }
  __syncthreads();

  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      al.load(p, ke, ra);
      bl.load(p, ke, rb);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      if constexpr (AK) af[i] = kfrag(As, wm + 16 * i);
      else af[i] = mnfrag<BM>(As, wm + 16 * i);
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      if constexpr (BKc) bfr[j] = kfrag(Bs, wn + 16 * j);
      else bfr[j] = mnfrag<BN>(Bs, wn + 16 * j);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if (more) {
      char* nxt = smem + (cur ^ 1) * STAGE;
      al.store(nxt, ra);
      bl.store(nxt + A_BYTES, rb);
      if constexpr (AK) al.advance(p); else al.advance(p, p.lda);
      if constexpr (BKc) bl.advance(p); else bl.advance(p, p.ldb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][e]: m = m0 + wm + 16i + (lane&15), n = n0 + wn + 16j + (lane>>4)*4 + e
  if (p.alpha_ptr) p.alpha *= *p.alpha_ptr;
  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  if constexpr (EPI == EPI_ATOMIC_F32) {
    // Stage the fp32 tile through LDS, half the rows at a time (the two
    // wave-rows take turns), then add it with atomics shaped as whole
    // contiguous row segments: every wave-instruction covers 64 consecutive
    // floats (256 B) of one row -- the full-rate atomic shape (MI355X_MICROARCH
    // "Global float atomics"); a 16-rows x 4-dwords shape runs ~17x slower.
    constexpr int HR = BM / 2;          // rows per half
    constexpr int FROW = BN + 4;        // fp32 row stride (pad: conflict-free b128 writes)
    static_assert(HR * FROW * 4 <= LDS, "atomic staging must fit the main-loop LDS");
    float* C = (float*)p.C;
    float* st = (float*)smem;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if ((wid >> 1) == half) {
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const int ml = 16 * i + lm;  // row within this half
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            const int nl = wn + 16 * j + ln4;
            *(f32x4*)(st + ml * FROW + nl) = acc[i][j] * p.alpha;
          }
        }
      }
      __syncthreads();
      constexpr int SEG = 64;                   // floats per wave-instruction
      constexpr int SEGS_PER_ROW = BN / SEG;    // 1 or 2
      for (int s = wid; s < HR * SEGS_PER_ROW; s += 4) {
        const int r = s / SEGS_PER_ROW, c = (s % SEGS_PER_ROW) * SEG + lane;
        const int m = m0 + half * HR + r, n = n0 + c;
        if (m < p.M && n < p.N) atomicAdd(C + (int64_t)m * p.ldc + n, st[r * FROW + c]);
      }
      __syncthreads();
    }
    return;
  } else if constexpr (EPI == EPI_F32) {
    float* C = (float*)p.C;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = m0 + wm + 16 * i + lm;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn + 16 * j + ln4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
          v[e] = act_fn(p.alpha * acc[i][j][e] + b, p.act);
          if (p.residual_f32 && n + e < p.N) v[e] += p.residual_f32[(int64_t)m * p.ldc + n + e];
        }
        float* dst = C + (int64_t)m * p.ldc + n;
        if (n + 4 <= p.N && (p.ldc & 3) == 0) {
          *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n + e < p.N) dst[e] = v[e];
        }
      }
    }
    return;
  } else {
    constexpr bool BNB = (EPI == EPI_BF16_BNB);
    // Stage bf16 tile in LDS (row stride CROW), then coalesced 16-B stores.
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int ml = wm + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int nl = wn + 16 * j + ln4;
        const int n = n0 + nl;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
          v[e] = act_fn(p.alpha * acc[i][j][e] + b, p.act);
        }
        u32x2 pk;
        pk[0] = pack_bf2(v[0], v[1]);
        pk[1] = pack_bf2(v[2], v[3]);
        *(u32x2*)(smem + ml * CROW + nl * 2) = pk;
      }
    }
    __syncthreads();
    constexpr int CPR = BN / 8, RPP = NT / CPR;
    const int c = tid % CPR, r0 = tid / CPR;
    const int n = n0 + c * 8;
    uint16_t* C = (uint16_t*)p.C;
    const bool vec = ((p.ldc & 7) == 0) && (n + 8 <= p.N);
    float s[8], ss[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
    float bsc[8], bsh[8], bmu[8];  // BN forward coefficients of this thread's 8 columns (EPI_BF16_BNB)
    if constexpr (BNB) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = min(n + e, p.N - 1);
        bsc[e] = p.st_coef[ch];
        bsh[e] = p.st_coef[p.N + ch];
        bmu[e] = p.st_coef[2 * p.N + ch];
      }
    }
    // Per-row finish: residual add, BN-backward partials / ReLU-mask (BNB) or BN-forward
    // partials, store.  Operands arrive pre-loaded (rv / xv / mb) so the fast path can
    // issue the loads of several rows before the first use.
    auto finish_row = [&](u32x4 v, const u32x4& rv, const u32x4& xv_raw, uint32_t mb, uint16_t* dst, bool vec_row) {
      if (p.residual) {
        float f[8], g[8];
        unpack8(v, f);
        unpack8(rv, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += g[e];
        v = pack8(f);
      }
      if (p.col_stats) {
        float f[8];
        unpack8(v, f);
        if constexpr (BNB) {  // (sum dz, sum dz*(x - mean)), dz = f * relu'(...)
          float xv[8];
          unpack8(xv_raw, xv);
          if (p.st_mask) {  // relu'(y) from the saved post-residual output's mask bits; store dz itself
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              f[e] = ((mb >> e) & 1u) ? f[e] : 0.f;
              s[e] += f[e];
              ss[e] += f[e] * (xv[e] - bmu[e]);
            }
            v = pack8(f);
          } else {  // relu'(x*scale + shift), recomputed from the pre-BN input
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dz = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
              s[e] += dz;
              ss[e] += dz * (xv[e] - bmu[e]);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] += f[e] * f[e]; }
        }
      }
      if (vec_row) {
        *(u32x4*)dst = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (n + e < p.N) dst[e] = (uint16_t)((e & 1) ? (v[e >> 1] >> 16) : (v[e >> 1] & 0xffff));
        }
      }
    };
    constexpr int RPI = BM / RPP;                 // rows per thread: 2, 4 or 8
    constexpr int G = RPI < 4 ? RPI : 4;          // rows whose operand loads are issued together
    const u32x4 z4 = zero16();
    if (vec && !p.g.remap && m0 + BM <= p.M) {
      // full tile, contiguous rows: G rows' residual / pre-BN / mask loads in flight at once
#pragma unroll
      for (int u0 = 0; u0 < RPI; u0 += G) {
        u32x4 tv[G], rv[G], xv[G];
        uint32_t mb[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int rr = r0 + (u0 + q) * RPP;
          const int64_t off = (int64_t)(m0 + rr) * p.ldc + n;
          tv[q] = *(const u32x4*)(smem + rr * CROW + c * 16);
          rv[q] = p.residual ? ld16(p.residual + off) : z4;
          xv[q] = (BNB && p.col_stats) ? ld16(p.st_x + off) : z4;
          mb[q] = (BNB && p.st_mask) ? (uint32_t)p.st_mask[off >> 3] : 0u;
        }
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int rr = r0 + (u0 + q) * RPP;
          finish_row(tv[q], rv[q], xv[q], mb[q], C + (int64_t)(m0 + rr) * p.ldc + n, true);
        }
      }
    } else {
      for (int rr = r0; rr < BM; rr += RPP) {
        const int m = m0 + rr;
        if (m >= p.M) break;
        const u32x4 v = *(const u32x4*)(smem + rr * CROW + c * 16);
        int64_t orow = m;
        if (p.g.remap) {  // phase dgrad: virtual row (n, hh, ww) -> real dX pixel
          // remap 1: dgrad-form geometry (virtual output = H x W); 2: forward-form (OH x OW)
          const int VW = p.g.remap == 2 ? p.g.OW : p.g.W, VH = p.g.remap == 2 ? p.g.OH : p.g.H;
          const int ww = m % VW, t = m / VW, hh = t % VH, nn = t / VH;
          orow = ((int64_t)nn * p.g.Hr + p.g.oa + p.g.psh * hh) * p.g.Wr + p.g.ob + p.g.psw * ww;
        }
        const int64_t off = orow * p.ldc + n;
        u32x4 rv = z4, xv = z4;
        uint32_t mb = 0;
        if (vec) {
          if (p.residual) rv = ld16(p.residual + off);
          if (BNB && p.col_stats) xv = ld16(p.st_x + off);
        } else {
          float g[8], xf[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            g[e] = (p.residual && n + e < p.N) ? bf2f(p.residual[off + e]) : 0.f;
            xf[e] = (BNB && p.col_stats && n + e < p.N) ? bf2f(p.st_x[off + e]) : 0.f;
          }
          rv = pack8(g);
          xv = pack8(xf);
        }
        if (BNB && p.st_mask) mb = p.st_mask[off >> 3];
        finish_row(v, rv, xv, mb, C + off, vec);
      }
    }
    if (p.col_stats) {
      // reduce over threads sharing column chunk c: lanes c + CPR*t within a wave, then 4 waves via LDS
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = CPR; o < 64; o <<= 1) {
          s[e] += __shfl_xor(s[e], o, 64);
          ss[e] += __shfl_xor(ss[e], o, 64);
        }
      }
      float* red = (float*)(smem + BM * CROW);  // [2][4 waves][BN]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[wid * BN + c * 8 + e] = s[e];
          red[4 * BN + wid * BN + c * 8 + e] = ss[e];
        }
      }
      __syncthreads();
      // per-(M-tile) partials, layout [2][N][tilesM]: no atomics, deterministic;
      // the BatchNorm finalize reduces the tilesM partials of each channel.
      if (tid < BN && n0 + tid < p.N) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) { a += red[w * BN + tid]; b += red[4 * BN + w * BN + tid]; }
        const int sld = p.stats_ld ? p.stats_ld : tilesM;
        p.col_stats[(int64_t)(n0 + tid) * sld + p.stats_off + tm] = a;
        p.col_stats[(int64_t)(p.N + n0 + tid) * sld + p.stats_off + tm] = b;
      }
    }
  }
}

template <int BM, int BN, int AL, int BL, int EPI>
static void launch_t(const IgemmArgs& a, int splits, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((igemm_kernel<BM, BN, AL, BL, EPI>), dim3(tiles * splits), dim3(NT), 0, st, a);
}

template <int AL, int BL, int EPI>
static int launch_tiles(const IgemmArgs& a, int bm, int bn, int splits, hipStream_t st) {
  if (bm == 128 && bn == 128) launch_t<128, 128, AL, BL, EPI>(a, splits, st);
  else if (bm == 128 && bn == 64) launch_t<128, 64, AL, BL, EPI>(a, splits, st);
  else if (bm == 64 && bn == 128) launch_t<64, 128, AL, BL, EPI>(a, splits, st);
  else if (bm == 64 && bn == 64) launch_t<64, 64, AL, BL, EPI>(a, splits, st);
  else return -2;
  return 0;
}

}  // namespace dpe

using namespace dpe;

// Supported (aload, bload, epi) combinations — one per GEMM role.
extern "C" int dpe_igemm_launch(const IgemmArgs* args, int bm, int bn, int aload, int bload, int epi, int splits,
                                hipStream_t st) {
  const IgemmArgs& a = *args;
  if (a.M <= 0 || a.N <= 0) return 0;
  if (splits < 1) splits = 1;
#define DPE_CASE(AL, BL, EP) \
  if (aload == AL && bload == BL && epi == EP) return launch_tiles<AL, BL, EP>(a, bm, bn, splits, st);
  // dense Linear / 1x1 conv
  DPE_CASE(A_DENSE_K, B_DENSE_K, EPI_BF16)
  DPE_CASE(A_DENSE_K, B_DENSE_K, EPI_F32)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_BF16)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_F32)
  DPE_CASE(A_DENSE_M, B_DENSE_N, EPI_ATOMIC_F32)
  DPE_CASE(A_DENSE_M, B_DENSE_N, EPI_F32)
  // conv
  DPE_CASE(A_CONV_FWD, B_DENSE_K, EPI_BF16)
  DPE_CASE(A_CONV_DGRAD, B_CONV_DGRAD, EPI_BF16)
  // data-grad feeding a BN+ReLU backward (partials from the epilogue)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_BF16_BNB)
  DPE_CASE(A_CONV_DGRAD, B_CONV_DGRAD, EPI_BF16_BNB)
  DPE_CASE(A_CONV_FWD, B_DENSE_K, EPI_BF16_BNB)
  DPE_CASE(A_DENSE_M, B_CONV_WGRAD, EPI_ATOMIC_F32)
#undef DPE_CASE
  return -1;
}
