// GEMMs for every 1x1 channel-mixing product of the WaveNet step:
//   skip    S  = Zcat·SKIPcat        (tmodel.py:171-184 summed over layers, tmodel.py:316-320)
//   head    H1 = relu(S)·POST1, logits = relu(H1)·POST2   (tmodel.py:187-215)
//   and their backward products (weight grads are split-K over the M = B·T positions).
// C[M][N] = epi( Σ_k A[m][k]·B[k][n] ).  A is stored either k-contiguous (A[m*lda+k]) or
// m-contiguous (A[k*lda+m]); B either n-contiguous (B[k*ldb+n]) or k-contiguous (B[n*ldb+k]).
// Two arithmetic forms (lbwn_gemm_set_mode): the default gemm_x3_kernel computes the f32
// products on the bf16 matrix cores by exact operand splitting (below); gemm_f32_kernel uses
// v_mfma_f32_32x32x2_f32.  In the latter the LDS image follows the global layout (no
// transposing stage), and the MFMA k-order is permuted so a k-contiguous operand feeds four
// MFMA steps from one ds_read_b128: at step j of an 8-deep group, lane half h uses k = 8g+4h+j.
#include <type_traits>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prologue.h"

namespace {

constexpr int NT = 256;
// padded row of an mn-contiguous image: fragment reads of lane halves h = 0/1 are rows 4 apart,
// and 4·(BMN+8) ≡ 32 (mod 64 banks) puts the halves on disjoint banks
constexpr int MNPAD = 8;

// BK = 16: the default (37 KB LDS, 2 blocks/CU).  BK = 8: the lean variant (21 KB) that fits
// beside a resident persistent chain block (131 KB) to run weight-gradient GEMMs concurrently.
template <bool KC, int BMN, int BK>
struct Stage {
  static constexpr int SREG = BK * BMN / (4 * NT);   // float4 staging registers per thread
  static constexpr int KCS = BK + 4;                 // padded k-contiguous row: conflict-free b128
  static constexpr int RS = BMN + MNPAD;             // row stride of the mn-contiguous image
  floatx4 v[SREG];
  static constexpr int LDS_FLOATS = KC ? BMN * KCS : BK * RS;

  LBWN_DEV void load(const float* __restrict__ P, long ld, int mn0, int MN, int k0, int K, int tid,
                     bool /*relu: applied in store()*/, const int* codes = nullptr) {
#pragma unroll
    for (int i = 0; i < SREG; ++i) {
      int r, c;  // r: index along M/N, c: along K
      if (KC) { r = tid / (BK / 4) + (NT / (BK / 4)) * i; c = (tid % (BK / 4)) * 4; }
      else    { c = tid / (BMN / 4) + (NT / (BMN / 4)) * i; r = (tid % (BMN / 4)) * 4; }
      int gr = mn0 + r, gk = k0 + c;
      floatx4 x = {0.f, 0.f, 0.f, 0.f};
      if (KC) {
        if (gr < MN && gk < K) x = *(const floatx4*)(P + (long)gr * ld + gk);
      } else if (codes) {
        if (gk < K) {
          const int cd = codes[gk] - gr;
          x[0] = cd == 0 ? 1.f : 0.f; x[1] = cd == 1 ? 1.f : 0.f;
          x[2] = cd == 2 ? 1.f : 0.f; x[3] = cd == 3 ? 1.f : 0.f;
        }
      } else {
        if (gk < K && gr < MN) x = *(const floatx4*)(P + (long)gk * ld + gr);
      }
      v[i] = x;   // relu (if any) is applied at store time: here it would force a vmcnt wait
    }
  }
  LBWN_DEV void store(float* lds, int tid, bool relu = false) {
#pragma unroll
    for (int i = 0; i < SREG; ++i) {
      if (relu) {
        v[i][0] = fmaxf(v[i][0], 0.f); v[i][1] = fmaxf(v[i][1], 0.f);
        v[i][2] = fmaxf(v[i][2], 0.f); v[i][3] = fmaxf(v[i][3], 0.f);
      }
      if (KC) {
        int r = tid / (BK / 4) + (NT / (BK / 4)) * i, c = (tid % (BK / 4)) * 4;
        *(floatx4*)(lds + r * KCS + c) = v[i];
      }
      else    { int c = tid / (BMN / 4) + (NT / (BMN / 4)) * i, r = (tid % (BMN / 4)) * 4; *(floatx4*)(lds + c * RS + r) = v[i]; }
    }
  }
  // fragment for rows [base, base+32) of group g: element j = value at k = 8g+4h+j
  LBWN_DEV floatx4 frag(const float* lds, int base, int g, int lane) const {
    int i = lane & 31, h = lane >> 5;
    if (KC) return *(const floatx4*)(lds + (base + i) * KCS + 8 * g + 4 * h);
    floatx4 f;
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = lds[(8 * g + 4 * h + j) * RS + base + i];
    return f;
  }
};

// XCD-aware bijective remap: blocks b and b+8 share an XCD under round-robin dispatch, so
// give each XCD a contiguous run of tiles (tiles sharing an A row-panel are adjacent).
LBWN_DEV int xcd_remap(int bid, int nwg) {
  int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Work item of this block over the whole (tiles × split-K) grid (grid = dim3(tiles, 1, splits)),
// k-split-major: one XCD runs every output tile of its k-slices together, so each slice's rows
// of both operands come from HBM into ONE L2 (per-z remapping spread a slice over all eight:
// ~3.4x the algorithmic bytes on dSKIP/dPOST1, profiles/pmc_traffic.json r01).
LBWN_DEV int gemm_work() { return xcd_remap(blockIdx.x + gridDim.x * blockIdx.z, gridDim.x * gridDim.z); }
LBWN_DEV int gemm_tile() { return gemm_work() % gridDim.x; }
LBWN_DEV int gemm_split() { return gemm_work() / gridDim.x; }
// 2-D blocking of a tm × tn tile grid over the 8 XCDs (no split-K): XCD x (= block % 8 under
// round-robin dispatch; placement is speed only) takes column half x & 1 and row quarter x >> 1,
// row-panel-major, so its L2 holds one half of the pre-split B (dZ: 2.45 of 4.9 MB) for the whole
// launch while A row panels stream through once per column half: A read twice and B eight halves,
// instead of B re-fetched per wave of row panels on every XCD (dZ 2.06x its algorithmic bytes,
// profiles/r04_pmc_read_requests.json)
LBWN_DEV int xcd2d_tile(int tm, int tn) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  if ((nwg & 7) || (tm & 3) || (tn & 1) || gridDim.z != 1 || nwg != tm * tn) return gemm_tile();
  const int x = bid & 7, j = bid >> 3, hn = tn >> 1, qm = tm >> 2;
  return ((x >> 1) * qm + j / hn) * tn + (x & 1) * hn + j % hn;
}

// Block tile BMT × BNT, 4 waves as 2 × 2, each wave (BMT/2) × (BNT/2) = MI × NI MFMA tiles.
// 128×128 tiles: four blocks (16 waves) per CU, i.e. at most 128 VGPRs; every register
// above that costs a wave per SIMD, and the k-loop needs that occupancy to hide its LDS reads
template <bool A_KC, bool B_KC, int BK, int BMT, int BNT>
__global__ __launch_bounds__(NT, (BMT * BNT > 128 * 128) ? 2 : 4) void gemm_f32_kernel(lbwn_gemm_args g) {
  constexpr int BM = BMT, BN = BNT, MI = BMT / 64, NI = BNT / 64;
  using SA = Stage<A_KC, BM, BK>;
  using SB = Stage<B_KC, BN, BK>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::LDS_FLOATS + SB::LDS_FLOATS)];
  auto As = [&](int i) { return smem + i * SA::LDS_FLOATS; };
  auto Bs = [&](int i) { return smem + 2 * SA::LDS_FLOATS + i * SB::LDS_FLOATS; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  const int t = gemm_tile();
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int kz0 = gemm_split() * g.k_per_split;
  const int kz1 = min(g.K, kz0 + g.k_per_split);
  const int ntiles = (kz1 - kz0 + BK - 1) / BK;

  floatx16 acc[MI][NI];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  SA sa;
  SB sb;
  if (ntiles > 0) {
    sa.load(g.A, g.lda, m0, g.M, kz0, kz1, tid, g.relu_a, g.a_codes);
    sb.load(g.B, g.ldb, n0, g.N, kz0, kz1, tid, false);
    sa.store(As(0), tid, g.relu_a);
    sb.store(Bs(0), tid);
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ntiles) {
      const int k0 = kz0 + (kt + 1) * BK;
      sa.load(g.A, g.lda, m0, g.M, k0, kz1, tid, g.relu_a, g.a_codes);
      sb.load(g.B, g.ldb, n0, g.N, k0, kz1, tid, false);
    }
#pragma unroll
    for (int gg = 0; gg < BK / 8; ++gg) {
      floatx4 fa[MI], fb[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) fa[mi] = sa.frag(As(cur), wm * (BM / 2) + mi * 32, gg, lane);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) fb[ni] = sb.frag(Bs(cur), wn * (BN / 2) + ni * 32, gg, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = mfma32(fa[mi][j], fb[ni][j], acc[mi][ni]);
    }
    if (kt + 1 < ntiles) {
      sa.store(As(cur ^ 1), tid, g.relu_a);
      sb.store(Bs(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // epilogue.  A 32×32 tile's mask values are loaded unconditionally at clamped indices before
  // any is used (a load under a per-row branch is waited for on its own: one memory round trip
  // per element, from HBM in the training step), then out-of-range rows / columns are skipped.
  const int h = lane >> 5, ci = lane & 31;
  float* C = g.C + (long)gemm_split() * g.split_stride;
  const bool raw = g.split_stride != 0;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + wn * (BN / 2) + ni * 32 + ci, colc = min(col, g.N - 1);
      const int rbase = m0 + wm * (BM / 2) + mi * 32;
      float mv[16];
      if (!raw && g.mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r) mv[r] = g.mask[(long)min(rbase + acc_row(r, h), g.M - 1) * g.ldm + colc];
      }
      const float bv = (!raw && g.bias) ? g.bias[colc] : 0.f;
      if (col >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + acc_row(r, h);
        float v = acc[mi][ni][r];
        if (!raw) {
          v += bv;
          if (g.relu_out) v = fmaxf(v, 0.f);
          if (g.mask && !(mv[r] > 0.f)) v = 0.f;
        }
        if (row < g.M) {
          if (!raw && g.accumulate) v += C[(long)row * g.ldc + col];
          C[(long)row * g.ldc + col] = v;
        }
      }
    }
}

// Σ over split slabs + epilogue; vectorised over n (N % 4 == 0).
__global__ void splitk_reduce_kernel(lbwn_gemm_args g, const float* __restrict__ slabs, int splits) {
  const long n4 = g.N / 4;
  const long total = (long)g.M * n4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = (int)(e / n4), col = (int)(e % n4) * 4;
    const float* src = slabs + (long)row * g.N + col;
    const long zs = (long)g.M * g.N;
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
    // 8 slabs per round, all loads issued before the first add (clamped, not predicated), summed
    // in slab order (deterministic)
    for (int z0 = 0; z0 < splits; z0 += 8) {
      floatx4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = *(const floatx4*)(src + (long)min(z0 + i, splits - 1) * zs);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (z0 + i < splits) s += v[i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = s[j];
      if (g.bias) v += g.bias[col + j];
      if (g.relu_out) v = fmaxf(v, 0.f);
      if (g.mask && !(g.mask[(long)row * g.ldm + col + j] > 0.f)) v = 0.f;
      float* c = g.C + (long)row * g.ldc + col + j;
      if (g.accumulate) v += *c;
      *c = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// f32 GEMM on the bf16 matrix cores by exact operand splitting.
// Every f32 x splits EXACTLY into three bf16 terms x = x0 + x1 + x2: x0 = RN(x) keeps 8
// significant bits, the f32 residual x - x0 is exact and holds ≤ 16 bits, x1 = RN(residual)
// takes 8 of them and the ≤ 8 left are x2, exactly (normal range; the data here is O(1)).
// a·b = Σ_{i,j} a_i·b_j; the six terms with i+j ≤ 2 are formed (each bf16 product is exact
// in f32) and accumulated in f32; the three dropped terms are ≤ 2·2^-27·|a·b|, below the
// 2^-24 rounding of every f32 accumulate.  So the result is an f32 GEMM (same operands,
// f32 accumulation, error class of the f32 MFMA chain: tests/test_gpu_parity.py
// ::test_gemm_split_accuracy) computed with 6 v_mfma_f32_32x32x16_bf16 (6 × 32 cycles) per
// 32×32×16 block instead of 8 v_mfma_f32_32x32x2_f32 (8 × 64 cycles): 2.67× the MFMA rate.
//
// Tile 128×128×32, 4 waves as 2×2 (64×64 each: 2×2 accumulators), two blocks per CU.  The
// operands are staged global f32 → registers (next k-step, issued before this step's MFMAs)
// → split → LDS as three bf16 planes per row: [row][plane][32 k] with a 208-B row
// (conflict-free b128 fragment reads: rows 52 dwords apart).  An mn-contiguous operand is
// transposed in registers (each thread loads a 4(k)×4(mn) block), so both layouts give the
// same k-contiguous image.  A weight operand can come pre-split (lbwn_gemm_args::b3, packed
// once per step by lbwn_split_planes_launch): its staging is a straight 16-B copy.
// Rows (m or n) past the end are read at a clamped row and never zeroed: they only feed
// output rows / columns that are discarded.  K past the end (K % 32 != 0) is zeroed.

constexpr int X3_BK = 32;
constexpr int X3_ROW = 104;               // bf16 per LDS row: 3 planes × 32 + 8 pad (208 B)
// gemm_x3q_kernel's rows (16x16x32 fragments: lane = (row l & 15, 16-B chunk l >> 4)): 224 B = 14
// 16-B slots, so every ds_read_b128 lane group ({0-3,12-15,20-27}, ... MI355X_MICROARCH.md §LDS)
// hits 16 distinct slots; at 208 B those reads were 2-way conflicted (PMC: 46 % of the kernel's
// LDS cycles were bank-conflict cycles)
constexpr int X3Q_ROW = 112;
constexpr int X3_NT = 256;
#ifndef X3_EXP
#define X3_EXP 0   // timing experiments only: 2 = one product per block, 4 = no in-loop global loads
#endif
#ifndef X3Q
#define X3Q 1        // the tall 128-column products on v_mfma_f32_16x16x32_bf16 (gemm_x3q_kernel)
#endif
#ifndef X3_OCC
#define X3_OCC 2
#endif
#ifndef X3R
#define X3R 1        // tall products with A k-contiguous and B pre-split: A in registers (gemm_x3r_kernel)
#endif

// split 4 consecutive-k values into the three planes and store them.  relu without a branch
// (a branch here split the k-step into basic blocks the scheduler cannot interleave with the
// MFMAs): as integers, max(bits, 0) is relu on f32 (negative floats are negative ints) and
// max(bits, INT_MIN) is the identity
LBWN_DEV void x3_store4(unsigned short* row, int k, floatx4 x, bool relu) {
  const int lo = relu ? 0 : (int)0x80000000;
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = __int_as_float(max(__float_as_int(x[j]), lo));
  unsigned h0, m0, l0, h1, m1, l1;
  split2((floatx2){x[0], x[1]}, h0, m0, l0);
  split2((floatx2){x[2], x[3]}, h1, m1, l1);
  const uintx2 h = {h0, h1}, m = {m0, m1}, l = {l0, l1};
  *(uintx2*)(row + k) = h;
  *(uintx2*)(row + 32 + k) = m;
  *(uintx2*)(row + 64 + k) = l;
}

// One f32 operand's k-step: ROWS rows × 32 k, NTHR threads.
// KC (k-contiguous in HBM): float4 i covers row (tid/8 + (NTHR/8)·i), k = 4·(tid%8).
// MN (mn-contiguous): 4(k)×4(mn) blocks b = tid + NTHR·q at k = 4·(b%8), mn = 4·(b/8); lanes
// with consecutive b%8 write one row's 64 B and rows 4 apart (≡ 16 banks): conflict-free.  When
// there are fewer blocks than threads (2·ROWS < NTHR), the extra waves load a duplicate and
// skip the store (wave-uniform).
// Row addresses are fixed per thread (set once); KFULL (K % 32 == 0): no per-step checks.
template <bool KC, bool KFULL, int ROWS, int NTHR, int RW = X3_ROW>
struct X3Stage {
  static constexpr int NQ = (2 * ROWS + NTHR - 1) / NTHR;          // MN: 4×4 blocks per thread
  static constexpr int NV = KC ? ROWS * 8 / NTHR : 4 * NQ;
  floatx4 v[2][NV];     // two payload sets (the 2-stage kernel keeps two k-steps in flight)
  const float* p[NV];   // KC: row pointers at the split's first k; MN: k-row pointers
  long step;            // floats per k-step
  int kq;               // 4·(tid%8): this thread's k offset in the step
  int kz;               // the split's first k
  unsigned okm[2];      // !KFULL: bit i = k in range (zeroed at store time, not at load)
  LBWN_DEV static bool mine(int tid, int q) { return KC || tid + NTHR * q < 2 * ROWS; }
  // gs: 0, or for a k-blocked operand (ld = 32, KFULL) the stride of its 32-deep k chunks (KC)
  // or of its 32-wide mn groups (MN)
  LBWN_DEV void init(const float* __restrict__ P, long ld, int mn0, int MN, int kz0, int tid, long gs = 0) {
    kq = 4 * (tid & 7);
    kz = kz0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (KC) {
        p[i] = P + (long)min(mn0 + (tid >> 3) + (NTHR / 8) * i, MN - 1) * ld +
               (gs ? (long)(kz0 / X3_BK) * gs : (long)kz0) + kq;
      } else {
        const int b = (tid + NTHR * (i >> 2)) % (2 * ROWS);
        const int mn = min(mn0 + 4 * (b >> 3), MN - 4);   // 4-aligned: never crosses a 32-group
        p[i] = P + (long)(kz0 + kq + (i & 3)) * ld + (gs ? (long)(mn >> 5) * gs + (mn & 31) : (long)mn);
      }
    }
    step = KC ? (gs ? gs : X3_BK) : X3_BK * ld;
  }
  // k-step t of the split ending at kend (kend read only when !KFULL); a clamped index keeps
  // every load unconditional
  template <int S = 0>
  LBWN_DEV void load(int t, int kend) {
    okm[S] = ~0u;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (KFULL) {
        v[S][i] = *(const floatx4*)(p[i] + t * step);
      } else {
        const int k = kz + t * X3_BK + kq + (KC ? 0 : (i & 3));       // this value's first k
        const int kc = KC ? min(k, kend - 4) : min(k, kend - 1);
        const long dk = kc - (kz + kq + (KC ? 0 : (i & 3)));           // k offset from p[i]
        v[S][i] = *(const floatx4*)(p[i] + (KC ? dk : dk * (step / X3_BK)));
        if (k >= kend) okm[S] &= ~(1u << i);
      }
    }
  }
  template <int S = 0>
  LBWN_DEV floatx4 val(int i) const {
    return (KFULL || ((okm[S] >> i) & 1)) ? v[S][i] : (floatx4){0.f, 0.f, 0.f, 0.f};
  }
  template <int S = 0>
  LBWN_DEV void store(unsigned short* lds, int tid, bool relu) {
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x3_store4(lds + ((tid >> 3) + (NTHR / 8) * i) * RW, kq, val<S>(i), relu);
    } else {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (!mine(tid, q)) continue;
        const int b = tid + NTHR * q;
        const floatx4 r0 = val<S>(4 * q), r1 = val<S>(4 * q + 1), r2 = val<S>(4 * q + 2), r3 = val<S>(4 * q + 3);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          floatx4 t = {r0[j], r1[j], r2[j], r3[j]};
          x3_store4(lds + (4 * (b >> 3) + j) * RW, kq, t, relu);
        }
      }
    }
  }
};

// Pre-split operand [rows][K/32][3][32] bf16: ROWS rows × 12 granules of 16 B per k-step.
template <int ROWS, int NTHR, int RW = X3_ROW>
struct X3Pre {
  static constexpr int NV = (ROWS * 12 + NTHR - 1) / NTHR;   // the last may be partial (whole waves)
  static_assert((ROWS * 12) % 64 == 0, "X3Pre: granules per wave");
  uintx4 v[2][NV];
  const unsigned short* p[NV];
  int ldst[NV];
  LBWN_DEV void init(const unsigned short* __restrict__ P3, int kchunks, int mn0, int MN, int kz0, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int gi = tid + NTHR * i, r = gi / 12, part = gi % 12;
      p[i] = P3 + ((long)min(mn0 + r, MN - 1) * kchunks + kz0 / X3_BK) * (3 * X3_BK) + 8 * part;
      ldst[i] = r * RW + 8 * part;
    }
  }
  template <int S = 0>
  LBWN_DEV void load(int t) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[S][i] = *(const uintx4*)(p[i] + t * (3 * X3_BK));
  }
  template <int S = 0>
  LBWN_DEV void store(unsigned short* lds) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if ((ROWS * 12) % NTHR == 0 || (int)threadIdx.x + NTHR * i < ROWS * 12) *(uintx4*)(lds + ldst[i]) = v[S][i];
  }
};

// Epilogue of a wave's 64×64 (2×2 accumulators) at (m0 + 64·wm, n0 + 64·wn): bias, relu, mask,
// accumulate; mask and C values loaded unconditionally at clamped indices before use.
// MI = 1 writes one 32-row band (rows m0 + 64·wm … +31) × 64 columns.
template <int MI>
LBWN_DEV void x3_epilogue_rows(const lbwn_gemm_args& g, floatx16 (&acc)[MI][2], int m0, int n0, int wm, int wn,
                               int lane, int nwm = 0, float* red = nullptr) {
  const int h = lane >> 5, ci = lane & 31;
  float* C = g.C + (long)gemm_split() * g.split_stride;
  const bool raw = g.split_stride != 0;
  float cs[2] = {0.f, 0.f};   // column partials (g.colpart) of this wave's 64-row band, lane half h
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int col = n0 + wn * 64 + ni * 32 + ci, colc = min(col, g.N - 1);
      const int rbase = m0 + wm * 64 + mi * 32;
      float mv[16], cv[16];
      if (!raw && g.mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r) mv[r] = g.mask[(long)min(rbase + acc_row(r, h), g.M - 1) * g.ldm + colc];
      }
      if (!raw && g.accumulate) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cv[r] = C[(long)min(rbase + acc_row(r, h), g.M - 1) * g.ldc + colc];
      }
      const float bv = (!raw && g.bias) ? g.bias[colc] : 0.f;
      if (col >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + acc_row(r, h);
        float v = acc[mi][ni][r];
        if (!raw) {
          v += bv;
          if (g.relu_out) v = fmaxf(v, 0.f);
          if (g.mask && !(mv[r] > 0.f)) v = 0.f;
          if (g.accumulate) v += cv[r];
        }
        if (row < g.M) {
          if (g.c_chain_ls)   // the chain's order: [col/32][row/32][(col/8)%4][row%32][(col/4)%2][4]
            C[(col >> 5) * g.c_chain_ls + ((((long)(row >> 5) * 4 + ((col >> 3) & 3)) * 32 + (row & 31)) * 8 + (col & 7))] = v;
          else
            C[(long)row * g.ldc + col] = v;
          cs[ni] += v;
        }
      }
    }
  // column partials of the block's 256 rows (4 waves along M): lane halves, then waves in a
  // fixed order through LDS (free after the k-loop's last barrier)
  if (MI == 2 && red && g.colpart && !raw) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      cs[ni] += __shfl_xor(cs[ni], 32);
      if (h == 0) red[wm * 128 + wn * 64 + ni * 32 + ci] = cs[ni];
    }
    __syncthreads();
    const int t = threadIdx.x, col = n0 + t;
    if (t < 128 && col < g.N) {
      float s = 0.f;
      for (int w = 0; w < nwm; ++w) s += red[w * 128 + t];
      g.colpart[(long)(m0 >> 8) * g.N + col] = s;
    }
  }
}
LBWN_DEV void x3_epilogue(const lbwn_gemm_args& g, floatx16 (&acc)[2][2], int m0, int n0, int wm, int wn, int lane,
                          int nwm, float* red) {
  x3_epilogue_rows<2>(g, acc, m0, n0, wm, wn, lane, nwm, red);
}

// Block tile (64·WM) × 128, WM × 2 waves of 64 × 64 (2 × 2 accumulators of 32 × 32).
// STAGES = 2: two LDS slots, one barrier per k-step; the next k-step's registers are split
// into the other slot between this step's two MFMA chunks, and the loads of the step after it
// are issued right behind (one k-step of load lead).
template <bool A_KC, bool B_KC, bool KFULL, bool BPRE, int WM, int STAGES>
__global__ __launch_bounds__(128 * WM, (WM == 2 && STAGES == 1) ? X3_OCC : 1) void gemm_x3_kernel(lbwn_gemm_args g) {
  constexpr int NTHR = 128 * WM, BM = 64 * WM, BN = 128, MI = 2, NI = 2;
  constexpr int SLOT = (BM + BN) * X3_ROW;
  __shared__ __attribute__((aligned(16))) unsigned short smem[STAGES * SLOT];
  unsigned short* sA = smem;
  unsigned short* sB = smem + BM * X3_ROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  if (g.step_advance && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && tid == 0)   // no-return atomic
    __hip_atomic_fetch_add(g.step_advance, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int t = gemm_tile();
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int kz0 = gemm_split() * g.k_per_split;
  const int kz1 = min(g.K, kz0 + g.k_per_split);
  const int ntiles = (kz1 - kz0 + X3_BK - 1) / X3_BK;

  floatx16 acc[MI][NI];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  X3Stage<A_KC, KFULL, BM, NTHR> sa;
  X3Stage<B_KC, KFULL, BN, NTHR> sb;
  X3Pre<BN, NTHR> sp;
  sa.init(g.A, g.lda, m0, g.M, kz0, tid, A_KC ? g.a_kstride : 0);
  if (BPRE) sp.init(g.b3, g.K / X3_BK, n0, g.N, kz0, tid);
  else sb.init(g.B, g.ldb, n0, g.N, kz0, tid, B_KC ? 0 : g.b_gstride);
  const bool relu_a = g.relu_a;
  if (ntiles > 0) {
    sa.load(0, kz1);
    if (BPRE) sp.load(0); else sb.load(0, kz1);
    sa.store(sA, tid, relu_a);
    if (BPRE) sp.store(sB); else sb.store(sB, tid, false);
  }
  __syncthreads();
  const int fi = lane & 31, fh = lane >> 5;
  const int fa_off = (wm * 64 + fi) * X3_ROW + 8 * fh, fb_off = (wn * 64 + fi) * X3_ROW + 8 * fh;

  // one 16-deep chunk c of the k-step held in slot `base`: 12 fragment reads, then 24 MFMAs
  using Frags = bf16x8[MI + NI][3];
  auto frags = [&](const unsigned short* base, int c, Frags& f) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) f[mi][p] = *(const bf16x8*)(base + fa_off + mi * 32 * X3_ROW + 32 * p + 16 * c);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        f[MI + ni][p] = *(const bf16x8*)(base + BM * X3_ROW + fb_off + ni * 32 * X3_ROW + 32 * p + 16 * c);
    }
  };
  auto mfmas = [&](const Frags& f) {
    // small terms first: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0
#pragma unroll
    for (int q = (X3_EXP == 2 ? 5 : 0); q < 6; ++q) {
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[mi][PA[q]], f[MI + ni][PB[q]], acc[mi][ni], 0, 0, 0);
    }
  };
  auto chunk = [&](const unsigned short* base, int c) {
    Frags f;
    frags(base, c, f);
    mfmas(f);
  };
  auto stage_store = [&](unsigned short* base) {
    sa.store(base, tid, relu_a);
    if (BPRE) sp.store(base + BM * X3_ROW); else sb.store(base + BM * X3_ROW, tid, false);
  };
  auto stage_load = [&](int k) {
    sa.load(k, kz1);
    if (BPRE) sp.load(k); else sb.load(k, kz1);
  };

  if (STAGES == 1) {
    for (int kt = 0; kt < ntiles; ++kt) {
      if (kt + 1 < ntiles && X3_EXP != 4) stage_load(kt + 1);
      chunk(smem, 0);
      chunk(smem, 1);
      if (kt + 1 < ntiles) {
        __syncthreads();
        stage_store(smem);
      }
      __syncthreads();
    }
  } else {
    // Two LDS slots and two register sets: k-step j's global loads land in set j & 1 two
    // k-steps ahead of its LDS store (a lead of ~2 k-steps of MFMA time against the L2/HBM
    // latency; one step of lead left the waves ~50 % parked on vmcnt): step 2.49 -> 2.41 ms
    // (same box, tools/gemm_ab.sh).  Reading chunk 1's fragments at the step start as well
    // (256 VGPRs) measured 2.53.  The prologue stored k-step 0 into slot 0 from set 0.
    // Every load and store of the loop is unconditional (k-steps past the end re-load the last
    // one, stores of them go to the idle slot): a guarded load made hipcc wait for all loads in
    // flight (its counts cannot assume the guarded ones were issued).
    const int last = max(ntiles - 1, 0);
    auto step = [&](int kt, auto sset) {
      constexpr int S = decltype(sset)::value;   // = (kt + 1) & 1: the slot written, the register set
      const unsigned short* cur = smem + (S ^ 1) * SLOT;   // compile-time slots: provably disjoint
      unsigned short* nxt = smem + S * SLOT;
      Frags f0, f1;
      frags(cur, 0, f0);
      mfmas(f0);
      sa.template store<S>(nxt, tid, relu_a);
      if (BPRE) sp.template store<S>(nxt + BM * X3_ROW); else sb.template store<S>(nxt + BM * X3_ROW, tid, false);
      const int kl = min(kt + 3, last);
      sa.template load<S>(kl, kz1);
      if (BPRE) sp.template load<S>(kl); else sb.template load<S>(kl, kz1);
      frags(cur, 1, f1);   // (before the stage stores: 2.40 -> 2.50 ms, same box)
      mfmas(f1);
      __syncthreads();
    };
    if (ntiles > 0) {
      sa.template load<1>(min(1, last), kz1);
      if (BPRE) sp.template load<1>(min(1, last)); else sb.template load<1>(min(1, last), kz1);
      sa.template load<0>(min(2, last), kz1);
      if (BPRE) sp.template load<0>(min(2, last)); else sb.template load<0>(min(2, last), kz1);
      int kt = 0;
      for (; kt + 1 < ntiles; kt += 2) {
        step(kt, std::integral_constant<int, 1>());
        step(kt + 1, std::integral_constant<int, 0>());
      }
      if (kt < ntiles) step(kt, std::integral_constant<int, 1>());
    }
  }

  x3_epilogue(g, acc, m0, n0, wm, wn, lane, WM, WM == 4 ? (float*)smem : nullptr);
}

// ---------------------------------------------------------------------------------------------
// 256 × 128 tiles with A in registers: A k-contiguous f32, B pre-split (lbwn_gemm_args::b3), the
// form of every tall product of the step (skip / post1 / post2 forward, dH1, dS, dZ).  Wave w owns
// rows m0 + 32w … +31 and all 128 columns (four 32 × 32 accumulators).  Lane (r, h) loads its own
// A values of each 32-deep k-step straight from global memory (row r, k = 8h … 8h+7 and
// 16+8h … 16+8h+7: two 32-B runs; a row's two lanes cover its 128-B line) and splits them in
// registers into exactly the MFMA fragments it supplies, so A never passes through the LDS: the
// LDS carries only B (26.6 KB per k-step instead of 80: no A image writes, no A fragment reads;
// B's fragment reads are the A reads' former count).  A two k-steps ahead and B three (two
// register sets each), one barrier per k-step.  The A fragments of k-step kt + 1 are split
// during k-step kt's MFMAs, so the split VALU fills MFMA gaps.
// Measured (skip fwd, M 32768 N 512 K 1600, same box, tools/gemm_exp.sh): 283-290 us against
// 290 for the LDS-staged gemm_x3_kernel<..., 4, 2>; MFMA busy 54 % at a 1.97 GHz clock
// (SQ_INSTS_MFMA·32 / SIMD vs GRBM_GUI_ACTIVE); timing-only ablations (wrong results): no
// barrier 273, no A split 268, line-coalesced A loads 274, no A loads 241, no B fragment reads
// 306 (the chip clocks down as the MFMAs pack closer: MI355X_MICROARCH.md 'DVFS give-back').
template <int NI>   // 4: 128 columns per tile; 3: 96 (N <= 96: arch5's dlc, N = 80)
__global__ __launch_bounds__(512, 1) void gemm_x3r_kernel(lbwn_gemm_args g) {
  constexpr int NTHR = 512, BM = 256, BN = 32 * NI;
  constexpr int SLOT = BN * X3_ROW;
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (g.N + BN - 1) / BN;
  if (g.step_advance && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && tid == 0)   // no-return atomic
    __hip_atomic_fetch_add(g.step_advance, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int t = gemm_tile();
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int kz0 = gemm_split() * g.k_per_split;
  const int kz1 = min(g.K, kz0 + g.k_per_split);
  const int ntiles = (kz1 - kz0) / X3_BK;   // K % 32 == 0 (pre-split B)
  const int last = max(ntiles - 1, 0);

  floatx16 acc[NI];
#pragma unroll
  for (int b = 0; b < NI; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  const float* pa = g.A + (long)min(m0 + 32 * wave + fr, g.M - 1) * g.lda + kz0 + 8 * fh;
  const int alo = g.relu_a ? 0 : (int)0x80000000;   // relu as an integer max (x3_store4)
  floatx4 av[2][4];
  auto a_load = [&](auto sset, int kt) {
    constexpr int S = decltype(sset)::value;
    const float* p = pa + kt * X3_BK;
    av[S][0] = *(const floatx4*)p;
    av[S][1] = *(const floatx4*)(p + 4);
    av[S][2] = *(const floatx4*)(p + 16);
    av[S][3] = *(const floatx4*)(p + 20);
  };
  // the three bf16x8 fragments of chunk c (k = 16c + 8h + j) from register set S
  auto a_split = [&](auto sset, int c, bf16x8 (&f)[3]) {
    constexpr int S = decltype(sset)::value;
    floatx4 x = av[S][2 * c], y = av[S][2 * c + 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = __int_as_float(max(__float_as_int(x[j]), alo));
      y[j] = __int_as_float(max(__float_as_int(y[j]), alo));
    }
    split8(x, y, f);
  };

  X3Pre<BN, NTHR> sp;
  sp.init(g.b3, g.K / X3_BK, n0, g.N, kz0, tid);
  if (ntiles > 0) {
    sp.load(0);
    sp.store(smem);
    a_load(std::integral_constant<int, 0>(), 0);
    a_load(std::integral_constant<int, 1>(), min(1, last));
    sp.template load<1>(min(1, last));
    sp.template load<0>(min(2, last));
  }
  __syncthreads();
  const int fb_off = fr * X3_ROW + 8 * fh;

  auto b_frags = [&](const unsigned short* base, int c, bf16x8 (&f)[NI][3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) f[ni][p] = *(const bf16x8*)(base + fb_off + ni * 32 * X3_ROW + 32 * p + 16 * c);
  };
  auto mfmas = [&](const bf16x8 (&fa)[3], const bf16x8 (&fb)[NI][3]) {
    // small terms first: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PA[q]], fb[ni][PB[q]], acc[ni], 0, 0, 0);
    }
  };
  bf16x8 fa[2][3];
  auto step = [&](int kt, auto sset) {
    constexpr int S = decltype(sset)::value;   // = (kt + 1) & 1
    const unsigned short* cur = smem + (S ^ 1) * SLOT;
    unsigned short* nxt = smem + S * SLOT;
    bf16x8 fn[2][3], fb[NI][3];
    b_frags(cur, 0, fb);
    mfmas(fa[0], fb);
    a_split(std::integral_constant<int, S>(), 0, fn[0]);
    a_split(std::integral_constant<int, S>(), 1, fn[1]);
    a_load(std::integral_constant<int, S>(), min(kt + 3, last));
    sp.template store<S>(nxt);
    sp.template load<S>(min(kt + 3, last));
    b_frags(cur, 1, fb);
    mfmas(fa[1], fb);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[c][p] = fn[c][p];
    __syncthreads();
  };
  if (ntiles > 0) {
    a_split(std::integral_constant<int, 0>(), 0, fa[0]);
    a_split(std::integral_constant<int, 0>(), 1, fa[1]);
    a_load(std::integral_constant<int, 0>(), min(2, last));
  }
  int kt = 0;
  for (; kt + 1 < ntiles; kt += 2) {
    step(kt, std::integral_constant<int, 1>());
    step(kt + 1, std::integral_constant<int, 0>());
  }
  if (kt < ntiles) step(kt, std::integral_constant<int, 1>());

  // epilogue (bias, relu, mask, accumulate, chain order, column partials): x3_epilogue_rows'
  // element rules on this wave's 32-row band × 128 columns
  const int h = fh, ci = fr;
  float* C = g.C + (long)gemm_split() * g.split_stride;
  const bool raw = g.split_stride != 0;
  const int rbase = m0 + 32 * wave;
  float cs[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    cs[ni] = 0.f;
    const int col = n0 + ni * 32 + ci, colc = min(col, g.N - 1);
    float mv[16], cv[16];
    if (!raw && g.mask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) mv[r] = g.mask[(long)min(rbase + acc_row(r, h), g.M - 1) * g.ldm + colc];
    }
    if (!raw && g.accumulate) {
#pragma unroll
      for (int r = 0; r < 16; ++r) cv[r] = C[(long)min(rbase + acc_row(r, h), g.M - 1) * g.ldc + colc];
    }
    const float bv = (!raw && g.bias) ? g.bias[colc] : 0.f;
    if (col >= g.N) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + acc_row(r, h);
      float v = acc[ni][r];
      if (!raw) {
        v += bv;
        if (g.relu_out) v = fmaxf(v, 0.f);
        if (g.mask && !(mv[r] > 0.f)) v = 0.f;
        if (g.accumulate) v += cv[r];
      }
      if (row < g.M) {
        if (g.c_chain_ls)
          C[(col >> 5) * g.c_chain_ls + ((((long)(row >> 5) * 4 + ((col >> 3) & 3)) * 32 + (row & 31)) * 8 + (col & 7))] = v;
        else
          C[(long)row * g.ldc + col] = v;
        cs[ni] += v;
      }
    }
  }
  if (g.colpart && !raw) {   // the block's 256-row column partials: lane halves, then waves in order
    float* red = (float*)smem;   // free after the k-loop's last barrier
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      cs[ni] += __shfl_xor(cs[ni], 32);
      if (h == 0) red[wave * BN + ni * 32 + ci] = cs[ni];
    }
    __syncthreads();
    const int col = n0 + tid;
    if (tid < BN && col < g.N) {
      float s = 0.f;
      for (int w = 0; w < 8; ++w) s += red[w * BN + tid];
      g.colpart[(long)(m0 >> 8) * g.N + col] = s;
    }
  }
}

// The same tile and data flow on v_mfma_f32_16x16x32_bf16 (equal cycles per FLOP; the chip holds a
// higher clock on it under load, MI355X_MICROARCH.md 'DVFS give-back' item 7): each wave's
// 32 × 128 band is 2 × 8 accumulators of 16 × 16, one MFMA takes the whole 32-deep k-step.  Lane
// l = (r = l & 15, q = l >> 4) supplies A[16mi + r][8q + j] (one 32-B run of a row per mi: a row's
// four lanes cover its 128-B line) and B[8q + j][16ni + r]; the k-step runs as two halves of 4
// column blocks.
// lane l <- lane l ^ 1 (CTRL 0xB1) or l ^ 2 (0x4E) within each quad: DPP quad_perm
template <int CTRL>
LBWN_DEV float quad_xor(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// AMN: the weight-gradient form (dSKIP, dPOST1, dPOST2: A and B both mn-contiguous, K = the
// positions): each lane loads its A fragment values as scalars -- per k row one 64-B run of 16
// consecutive rows i, the same bytes as the k-contiguous form's two 32-B runs -- and splits them in
// registers as above (A never passes through the LDS); B is staged like the LDS-staged kernel's
// mn-contiguous operand (4(k) x 4(n) blocks transposed in registers, split, written as planes).
template <int NB, bool AMN = false>   // 16-column blocks: 8 (128 columns), 10 (160: dZ's N = 1600) or 6 (96: N <= 96, arch5's dlc)
__global__ __launch_bounds__(512, 1) void gemm_x3q_kernel(lbwn_gemm_args g) {
  // the k-step's column blocks run in NP parts of NH (B fragments live for one part: NB = 10 in
  // two parts of 5 spilled 32 VGPRs)
  constexpr int NP = NB == 10 ? 5 : 2;
  constexpr int NTHR = 512, BM = 256, BN = 16 * NB, NH = NB / NP;
  constexpr int SLOT = BN * X3Q_ROW;
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (g.N + BN - 1) / BN;
  if (g.step_advance && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && tid == 0)   // no-return atomic
    __hip_atomic_fetch_add(g.step_advance, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int t = (NB == 10 && g.xcd2d) ? xcd2d_tile((g.M + BM - 1) / BM, tiles_n) : gemm_tile();
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  // a consumer's mask-bit word (mbits), loaded now: one 8-B load whose latency the k-loop hides
  const long mw = ((long)t * 8 + wave) * 64 + lane;
  // (the k-contiguous form only: in the AMN form, dSKIP's, they cost 8 VGPRs -- 240 -> 248, which
  // left no room beside it for the side stream's dPRE scatter: 80 -> 297 us, step +40 us)
  constexpr bool MB = NB == 8 && !AMN;
  const bool bits_in = MB && g.split_stride == 0 && g.mbits, bits_out = MB && g.split_stride == 0 && g.mbits_out;
  const unsigned long long mbr = bits_in ? g.mbits[mw] : 0ull;
  const int kz0 = gemm_split() * g.k_per_split;
  const int kz1 = min(g.K, kz0 + g.k_per_split);
  const int ntiles = (kz1 - kz0) / X3_BK;   // K % 32 == 0 (pre-split B; AMN: checked by the launcher)
  const int last = max(ntiles - 1, 0);

  floatx4 acc[2][NB];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = (floatx4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const long aks = g.a_kstride ? g.a_kstride : X3_BK;   // floats per 32-deep k-step of A
  // (AMN with a_gstride: the wave's 32 rows are one 32-row group, clamped whole into the matrix)
  const int ag0 = min(m0 + 32 * wave, max((g.M - 1) & ~31, 0));
  const float* pa0 = AMN ? (g.a_gstride ? g.A + (ag0 >> 5) * g.a_gstride + fr + (long)(kz0 + 8 * fq) * 32
                                        : g.A + min(m0 + 32 * wave + fr, g.M - 1) + (long)(kz0 + 8 * fq) * g.lda)
                         : g.A + (long)min(m0 + 32 * wave + fr, g.M - 1) * g.lda + (kz0 / X3_BK) * aks + 8 * fq;
  const float* pa1 = AMN ? (g.a_gstride ? pa0 + 16
                                        : g.A + min(m0 + 32 * wave + 16 + fr, g.M - 1) + (long)(kz0 + 8 * fq) * g.lda)
                         : g.A + (long)min(m0 + 32 * wave + 16 + fr, g.M - 1) * g.lda + (kz0 / X3_BK) * aks + 8 * fq;
  const int alo = g.relu_a ? 0 : (int)0x80000000;   // relu as an integer max (x3_store4)
  floatx4 av[2][4];
  auto a_load = [&](auto sset, int kt) {
    constexpr int S = decltype(sset)::value;
    if (AMN) {   // A[i][k] at A[k·lda + i]: k rows 32kt + 8fq + j
      const long ko = (long)kt * X3_BK * g.lda;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[S][j >> 2][j & 3] = pa0[ko + j * g.lda];
        av[S][2 + (j >> 2)][j & 3] = pa1[ko + j * g.lda];
      }
    } else if (NB == 10) {
      // dZ: A row panels non-temporal, so that the 6.4 panels in flight per XCD do not evict the
      // B half its L2 keeps for the launch (xcd2d_tile)
      av[S][0] = __builtin_nontemporal_load((const floatx4*)(pa0 + kt * aks));
      av[S][1] = __builtin_nontemporal_load((const floatx4*)(pa0 + kt * aks + 4));
      av[S][2] = __builtin_nontemporal_load((const floatx4*)(pa1 + kt * aks));
      av[S][3] = __builtin_nontemporal_load((const floatx4*)(pa1 + kt * aks + 4));
    } else {
      av[S][0] = *(const floatx4*)(pa0 + kt * aks);
      av[S][1] = *(const floatx4*)(pa0 + kt * aks + 4);
      av[S][2] = *(const floatx4*)(pa1 + kt * aks);
      av[S][3] = *(const floatx4*)(pa1 + kt * aks + 4);
    }
  };
  auto a_split = [&](auto sset, int mi, bf16x8 (&f)[3]) {
    constexpr int S = decltype(sset)::value;
    floatx4 x = av[S][2 * mi], y = av[S][2 * mi + 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = __int_as_float(max(__float_as_int(x[j]), alo));
      y[j] = __int_as_float(max(__float_as_int(y[j]), alo));
    }
    split8(x, y, f);
  };

  // B: pre-split planes copied to LDS, or (AMN) an mn-contiguous f32 operand split on the way
  X3Pre<BN, NTHR, X3Q_ROW> sp;
  X3Stage<false, true, BN, NTHR, X3Q_ROW> sm_b;
  auto b_load = [&](auto sset, int kt) {
    constexpr int S = decltype(sset)::value;
    if (AMN) sm_b.template load<S>(kt, 0);
    else sp.template load<S>(kt);
  };
  auto b_store = [&](auto sset, unsigned short* lds) {
    constexpr int S = decltype(sset)::value;
    if (AMN) sm_b.template store<S>(lds, tid, false);
    else sp.template store<S>(lds);
  };
  if (AMN) sm_b.init(g.B, g.ldb, n0, g.N, kz0, tid);
  else sp.init(g.b3, g.K / X3_BK, n0, g.N, kz0, tid);
  if (ntiles > 0) {
    b_load(std::integral_constant<int, 0>(), 0);
    b_store(std::integral_constant<int, 0>(), smem);
    a_load(std::integral_constant<int, 0>(), 0);
    a_load(std::integral_constant<int, 1>(), min(1, last));
    b_load(std::integral_constant<int, 1>(), min(1, last));
    b_load(std::integral_constant<int, 0>(), min(2, last));
  }
  __syncthreads();
  const int fb_off = fr * X3Q_ROW + 8 * fq;

  auto b_frags = [&](const unsigned short* base, int half, bf16x8 (&f)[NH][3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int nb = 0; nb < NH; ++nb) f[nb][p] = *(const bf16x8*)(base + fb_off + (NH * half + nb) * 16 * X3Q_ROW + 32 * p);
  };
  auto mfmas = [&](const bf16x8 (&fa)[2][3], const bf16x8 (&fb)[NH][3], int half) {
    // small terms first: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0
#pragma unroll
    for (int qq = 0; qq < 6; ++qq) {
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nb = 0; nb < NH; ++nb)
          acc[mi][NH * half + nb] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][PA[qq]], fb[nb][PB[qq]], acc[mi][NH * half + nb], 0, 0, 0);
    }
  };
  bf16x8 fa[2][3];
  auto step = [&](int kt, auto sset) {
    constexpr int S = decltype(sset)::value;   // = (kt + 1) & 1
    const unsigned short* cur = smem + (S ^ 1) * SLOT;
    unsigned short* nxt = smem + S * SLOT;
    bf16x8 fn[2][3], fb[NH][3];
    b_frags(cur, 0, fb);
    mfmas(fa, fb, 0);
    a_split(std::integral_constant<int, S>(), 0, fn[0]);
    a_split(std::integral_constant<int, S>(), 1, fn[1]);
    a_load(std::integral_constant<int, S>(), min(kt + 3, last));
    b_store(std::integral_constant<int, S>(), nxt);
    b_load(std::integral_constant<int, S>(), min(kt + 3, last));
#pragma unroll
    for (int part = 1; part < NP; ++part) {
      b_frags(cur, part, fb);
      mfmas(fa, fb, part);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[c][p] = fn[c][p];
    __syncthreads();
  };
  if (ntiles > 0) {
    a_split(std::integral_constant<int, 0>(), 0, fa[0]);
    a_split(std::integral_constant<int, 0>(), 1, fa[1]);
    a_load(std::integral_constant<int, 0>(), min(2, last));
  }
  int kt = 0;
  for (; kt + 1 < ntiles; kt += 2) {
    step(kt, std::integral_constant<int, 1>());
    step(kt + 1, std::integral_constant<int, 0>());
  }
  if (kt < ntiles) step(kt, std::integral_constant<int, 1>());

  // epilogue: element (mi, nb, i) is row rbase + 16mi + 4q + i, column n0 + 16nb + r
  float* C = g.C + (long)gemm_split() * g.split_stride;
  const bool raw = g.split_stride != 0;
  const int rbase = m0 + 32 * wave;
  float cs[NB];
  if (g.c_chain_ls && !raw) {
    // dZ in the chain's order (no bias / mask / accumulate): a 4x4 transpose among lanes fr&3
    // (two xor exchanges) gives each lane one row x 4 consecutive columns = one 16-B run of the
    // destination; stored write-through (sc1): the 210-MB output streams past the L2 instead of
    // evicting the B half it holds (xcd2d_tile)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      cs[nb] = 0.f;
      const int col0 = n0 + nb * 16;
      if (col0 >= g.N) continue;   // wave-uniform
      const long chunk = g.c_chain_ls * 4;
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
          C + (long)(col0 >> 5) * g.c_chain_ls, (short)0, (int)(chunk < 0x7fffffffL ? chunk : 0x7fffffffL), 0x00020000);
      const int c = fr & 3, colq = col0 + 4 * (fr >> 2);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        float a0 = acc[mi][nb][0], a1 = acc[mi][nb][1], a2 = acc[mi][nb][2], a3 = acc[mi][nb][3];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (rbase + 16 * mi + 4 * fq + e < g.M) cs[nb] += acc[mi][nb][e];
        const bool odd = c & 1, hi = c & 2;
        {   // lane xor 1 / xor 2 within the quad: DPP quad_perm (VALU) instead of ds_bpermute
          const float r0 = quad_xor<0xB1>(odd ? a0 : a1), r1 = quad_xor<0xB1>(odd ? a2 : a3);
          if (odd) { a0 = r0; a2 = r1; } else { a1 = r0; a3 = r1; }
        }
        {
          const float q0 = quad_xor<0x4E>(hi ? a0 : a2), q1 = quad_xor<0x4E>(hi ? a1 : a3);
          if (hi) { a0 = q0; a1 = q1; } else { a2 = q0; a3 = q1; }
        }
        const int row = rbase + 16 * mi + 4 * fq + c;
        const int off = row < g.M ? (int)(((((long)(row >> 5) * 4 + ((colq >> 3) & 3)) * 32 + (row & 31)) * 8 + (colq & 7)) * 4)
                                  : 0x7ffffff0;   // past the record: dropped
        __builtin_amdgcn_raw_buffer_store_b128((floatx4){a0, a1, a2, a3}, rc, off, 0, 16);
      }
    }
  } else if (!g.accumulate && (g.ldc & 3) == 0 && (g.N & 3) == 0 && !((uintptr_t)C & 15)) {
    // row-major C: the elementwise epilogue per element, then the dZ path's 4x4 quad transpose so
    // that each lane stores one row x 4 consecutive columns as one 16-B store (64 single-float
    // stores per lane before)
    unsigned long long mbw = 0ull;
    const int c = fr & 3;
    const bool odd = c & 1, hi = c & 2;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      cs[nb] = 0.f;
      const int col0 = n0 + nb * 16;
      if (col0 >= g.N) continue;   // wave-uniform
      const int col = col0 + fr, colc = min(col, g.N - 1);
      float mv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int rowc = min(rbase + 16 * (e >> 2) + 4 * fq + (e & 3), g.M - 1);
        if (!raw && g.mask && !bits_in) mv[e] = g.mask[(long)rowc * g.ldm + colc];
      }
      const float bv = (!raw && g.bias) ? g.bias[colc] : 0.f;
      float vv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int row = rbase + 16 * (e >> 2) + 4 * fq + (e & 3);
        float v = acc[e >> 2][nb][e & 3];
        if (!raw) {
          v += bv;
          if (g.relu_out) v = fmaxf(v, 0.f);
          if (bits_in) {
            if (!((mbr >> (8 * nb + e)) & 1ull)) v = 0.f;
          } else if (g.mask && !(mv[e] > 0.f)) {
            v = 0.f;
          }
          if (bits_out && v > 0.f) mbw |= 1ull << (8 * nb + e);
        }
        vv[e] = v;
        if (col < g.N && row < g.M) cs[nb] += v;
      }
      const int colq = col0 + 4 * (fr >> 2);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        float a0 = vv[4 * mi], a1 = vv[4 * mi + 1], a2 = vv[4 * mi + 2], a3 = vv[4 * mi + 3];
        {
          const float r0 = quad_xor<0xB1>(odd ? a0 : a1), r1 = quad_xor<0xB1>(odd ? a2 : a3);
          if (odd) { a0 = r0; a2 = r1; } else { a1 = r0; a3 = r1; }
        }
        {
          const float q0 = quad_xor<0x4E>(hi ? a0 : a2), q1 = quad_xor<0x4E>(hi ? a1 : a3);
          if (hi) { a0 = q0; a1 = q1; } else { a2 = q0; a3 = q1; }
        }
        const int row = rbase + 16 * mi + 4 * fq + c;
        if (row < g.M && colq < g.N) *(floatx4*)(C + (long)row * g.ldc + colq) = (floatx4){a0, a1, a2, a3};
      }
    }
    if (bits_out) g.mbits_out[mw] = mbw;
  } else {
  unsigned long long mbw = 0ull;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    cs[nb] = 0.f;
    const int col = n0 + nb * 16 + fr, colc = min(col, g.N - 1);
    float mv[8], cv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int rowc = min(rbase + 16 * (e >> 2) + 4 * fq + (e & 3), g.M - 1);
      if (!raw && g.mask && !bits_in) mv[e] = g.mask[(long)rowc * g.ldm + colc];
      if (!raw && g.accumulate) cv[e] = C[(long)rowc * g.ldc + colc];
    }
    const float bv = (!raw && g.bias) ? g.bias[colc] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int row = rbase + 16 * (e >> 2) + 4 * fq + (e & 3);
      float v = acc[e >> 2][nb][e & 3];
      if (!raw) {
        v += bv;
        if (g.relu_out) v = fmaxf(v, 0.f);
        if (bits_in) {
          if (!((mbr >> (8 * nb + e)) & 1ull)) v = 0.f;
        } else if (g.mask && !(mv[e] > 0.f)) {
          v = 0.f;
        }
        if (bits_out && v > 0.f) mbw |= 1ull << (8 * nb + e);
        if (g.accumulate) v += cv[e];
      }
      if (col >= g.N) continue;
      if (row < g.M) {
        if (g.c_chain_ls)
          C[(col >> 5) * g.c_chain_ls + ((((long)(row >> 5) * 4 + ((col >> 3) & 3)) * 32 + (row & 31)) * 8 + (col & 7))] = v;
        else
          C[(long)row * g.ldc + col] = v;
        cs[nb] += v;
      }
    }
  }
  if (bits_out) g.mbits_out[mw] = mbw;
  }
  if (g.colpart && !raw) {   // the block's 256-row column partials: lane quarters, then waves in order
    float* red = (float*)smem;   // free after the k-loop's last barrier
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      cs[nb] += __shfl_xor(cs[nb], 16);
      cs[nb] += __shfl_xor(cs[nb], 32);
      if (fq == 0) red[wave * BN + nb * 16 + fr] = cs[nb];
    }
    __syncthreads();
    const int col = n0 + tid;
    if (tid < BN && col < g.N) {
      float s = 0.f;
      for (int w = 0; w < 8; ++w) s += red[w * BN + tid];
      g.colpart[(long)(m0 >> 8) * g.N + col] = s;
    }
  }
}

// Pre-split planes of the weights (body and SplitJobs in prologue.h; blockIdx.y = job)
static_assert(PLANE_BK == X3_BK, "pre-split chunk = GEMM k-step");
__global__ void split_planes_kernel(SplitJobs jb) { split_planes_body(jb, blockIdx.y, blockIdx.x, gridDim.x); }

}  // namespace

namespace {
// shape checks and split-K set-up shared by both GEMM forms
int gemm_setup(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int& split_k, float* slab_ws, int BK,
               int BM, int BN, lbwn_gemm_args& g, dim3& grid) {
  LBWN_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0, "gemm: empty shape M=%d N=%d K=%d", a.M, a.N, a.K);
  LBWN_REQUIRE(a.K % 4 == 0 || !a_kcontig, "gemm: K %% 4 != 0 with k-contiguous A");
  LBWN_REQUIRE(a.K % 4 == 0 || !b_kcontig, "gemm: K %% 4 != 0 with k-contiguous B");
  LBWN_REQUIRE(a.M % 4 == 0 || a_kcontig, "gemm: M %% 4 != 0 with m-contiguous A");
  LBWN_REQUIRE(a.N % 4 == 0, "gemm: N %% 4 != 0");
  LBWN_REQUIRE(a.lda % 4 == 0 && a.ldb % 4 == 0, "gemm: lda/ldb must be multiples of 4");
  LBWN_REQUIRE(a.a_codes == nullptr || !a_kcontig, "gemm: one-hot A must be m-contiguous");
  LBWN_REQUIRE((a.a_codes || (((uintptr_t)a.A) & 15) == 0) && (((uintptr_t)a.B) & 15) == 0,
               "gemm: A/B not 16-B aligned");
  LBWN_REQUIRE(!a.a_kstride || (a_kcontig && a.lda == 32 && a.K % 32 == 0 && !a.a_codes && lbwn_gemm_mode() == 1),
               "gemm: k-blocked A needs k-contiguous A, lda = 32, K %% 32 == 0 and the bf16-split form");
  LBWN_REQUIRE(!a.b_gstride || (!b_kcontig && a.ldb == 32 && !a.b3 && lbwn_gemm_mode() == 1),
               "gemm: mn-blocked B needs mn-contiguous B, ldb = 32, no pre-split and the bf16-split form");
  LBWN_REQUIRE(!a.a_gstride || (!a_kcontig && a.lda == 32 && !b_kcontig && !a.b_gstride && !a.b3 && a.M >= 256 &&
                                a.K % 32 == 0 && !a.mask && !a.bias && !a.colpart && !a.c_chain_ls && !a.a_codes &&
                                lbwn_gemm_mode() == 1),
               "gemm: mn-blocked A needs the AMN weight-gradient form (lda = 32, M >= 256, K %% 32 == 0)");
  if (split_k < 1) split_k = 1;
  g = a;
  int kps = (a.K + split_k - 1) / split_k;
  kps = (kps + BK - 1) / BK * BK;
  split_k = (a.K + kps - 1) / kps;
  g.k_per_split = kps;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  grid = dim3(tiles, 1, split_k);
  if (split_k > 1) {
    LBWN_REQUIRE(slab_ws != nullptr, "gemm: split-K needs a slab workspace");
    g.C = slab_ws;
    g.ldc = a.N;
    g.split_stride = (long)a.M * a.N;
  } else {
    g.split_stride = 0;
  }
  return 0;
}

int splitk_finish(const lbwn_gemm_args& a, int split_k, const float* slab_ws, hipStream_t st) {
  if (a.splits_deferred) {   // the consumer sums the partials itself (lc_up_bwd_kernel)
    LBWN_REQUIRE(!a.bias && !a.relu_out && !a.mask && !a.accumulate, "gemm: deferred split-K needs a plain product");
    *a.splits_deferred = split_k;
    return 0;
  }
  if (split_k > 1) {
    const long total = (long)a.M * (a.N / 4);
    int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(a, slab_ws, split_k);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}

template <bool KFULL, bool BPRE, int WM>
int gemm_launch_x3_t(const lbwn_gemm_args& g, const dim3& grid, int a_kcontig, int b_kcontig, hipStream_t st) {
  constexpr int NTHR = 128 * WM, S = WM == 4 ? 2 : 1;
  if (BPRE) {
    if (a_kcontig) gemm_x3_kernel<true, true, KFULL, true, WM, S><<<grid, NTHR, 0, st>>>(g);
    else gemm_x3_kernel<false, true, KFULL, true, WM, S><<<grid, NTHR, 0, st>>>(g);
  } else if (a_kcontig && b_kcontig) gemm_x3_kernel<true, true, KFULL, false, WM, S><<<grid, NTHR, 0, st>>>(g);
  else if (a_kcontig) gemm_x3_kernel<true, false, KFULL, false, WM, S><<<grid, NTHR, 0, st>>>(g);
  else if (b_kcontig) gemm_x3_kernel<false, true, KFULL, false, WM, S><<<grid, NTHR, 0, st>>>(g);
  else gemm_x3_kernel<false, false, KFULL, false, WM, S><<<grid, NTHR, 0, st>>>(g);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int gemm_launch_x3(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws,
                   hipStream_t st) {
  LBWN_REQUIRE(a.a_codes == nullptr, "gemm (bf16 split): one-hot A not supported");
  LBWN_REQUIRE(a.colpart == nullptr || split_k <= 1, "gemm (bf16 split): column partials need split_k = 1");
  LBWN_REQUIRE(!a.c_chain_ls || (split_k <= 1 && !a.accumulate && !a.mask && a.N % 32 == 0 &&
                                 a.c_chain_ls >= (a.M + 31L) / 32 * 32 * 32),
               "gemm (bf16 split): chain-order C needs split_k = 1, no accumulate/mask, N %% 32 == 0");
  LBWN_REQUIRE(a.b3 == nullptr || (a.K % X3_BK == 0 && (((uintptr_t)a.b3) & 15) == 0),
               "gemm (bf16 split): pre-split B needs K %% 32 == 0 and 16-B alignment");
  LBWN_REQUIRE(!(a.mbits || a.mbits_out) ||
                   (lbwn_gemm_x3q8_form(a.M, a.N, a.K, a_kcontig, a.b3 != nullptr, a.row_exact, a.colpart != nullptr) &&
                    split_k <= 1),
               "gemm (bf16 split): mask bits need the gemm_x3q_kernel<8> form without split-K");
  // 256-row tiles (8 waves, 2-stage pipeline) for the tall k-contiguous products with N <= 2048
  // (skip fwd, post1/post2 fwd, dH1, dS: 3-8 % faster; dZ, N = 1600: step -0.5 % in a same-box
  // A/B since the epilogue and split changes); 128-row tiles at 2 blocks per CU for the rest
  // (the mn-contiguous weight gradients: 1.3-1.5x slower on 256-row tiles)
  // (256-row tiles for dSKIP too, with the 2-deep staging: 341 -> 476 us)
  const int wm = (a.colpart || (a_kcontig && a.N <= 2048 && (a.M >= 8192 || a.row_exact))) ? 4 : 2;
  lbwn_gemm_args g;
  dim3 grid;
  int e = gemm_setup(a, a_kcontig, b_kcontig, split_k, slab_ws, X3_BK, 64 * wm, 128, g, grid);
  if (e) return e;
  const bool kfull = a.K % X3_BK == 0, pre = a.b3 != nullptr;
  if (X3Q && !a_kcontig && !b_kcontig && kfull && !pre && !a.mask && !a.bias && !a.colpart && !a.c_chain_ls &&
      !a.b_gstride && a.M >= 256 && a.N % 4 == 0 && (((a.M + 255) / 256) * ((a.N + 127) / 128) >= 8 || a.a_gstride)) {
    // the weight-gradient products with >= 8 output tiles (dSKIP, dPOST1): 256 x 128 tiles with A
    // in registers (gemm_x3q_kernel AMN).  tools/gemm_bench.py, same box: dSKIP split 9 315 vs
    // 355 us, dPOST1 split 32 97 vs 107; dPOST2 (4 tiles) 87 vs 77 stays on the 2-per-CU kernel.
    // N <= 96 (dLCcat as DVᵀ·lc, N = n_lc_out): 96-column tiles
    if ((e = gemm_setup(a, a_kcontig, b_kcontig, split_k, slab_ws, X3_BK, 256, a.N <= 96 ? 96 : 128, g, grid))) return e;
    if (a.N <= 96) gemm_x3q_kernel<6, true><<<grid, 512, 0, st>>>(g);
    else gemm_x3q_kernel<8, true><<<grid, 512, 0, st>>>(g);
    LBWN_CHECK_LAUNCH();
    return splitk_finish(a, split_k, slab_ws, st);
  }
  // every other kernel below reads A row-major: an mn-blocked A (a_gstride) would be read in the
  // wrong layout there
  LBWN_REQUIRE(!a.a_gstride, "gemm: mn-blocked A (a_gstride) needs the AMN A-in-registers form (X3Q, no pre-split B, "
                             "no epilogue, M >= 256)");
  if (wm == 4 && X3R && kfull && pre && a_kcontig) {
    if (a.N <= 96) {   // 96-column tiles: the grid is re-formed for them
      grid.x = (unsigned)(((a.M + 255) / 256) * ((a.N + 95) / 96));
      if (X3Q) gemm_x3q_kernel<6><<<grid, 512, 0, st>>>(g);
      else gemm_x3r_kernel<3><<<grid, 512, 0, st>>>(g);
    } else if (X3Q && a.N % 160 == 0 && a.N > 512) {
      // N = 1600 (dZ): 160-column tiles, so the grid is whole rounds of 256 blocks (M/256 x 10 at
      // C2 = 1280 = 5 rounds) instead of 128-column ones (13 column tiles, the last half empty:
      // 1664 = 6.5 rounds; same box 2.296-2.304 vs 2.342-2.353 ms per step).
      // a.xcd2d (the caller's choice): the 2-D XCD blocking of the tiles (xcd2d_tile)
      grid.x = (unsigned)(((a.M + 255) / 256) * (a.N / 160));
      gemm_x3q_kernel<10><<<grid, 512, 0, st>>>(g);
    } else if (X3Q) {   // (lbwn_gemm_x3q8_form)
      gemm_x3q_kernel<8><<<grid, 512, 0, st>>>(g);
    } else {
      gemm_x3r_kernel<4><<<grid, 512, 0, st>>>(g);
    }
    LBWN_CHECK_LAUNCH();
  } else if (wm == 4) {
    if (kfull && pre) e = gemm_launch_x3_t<true, true, 4>(g, grid, a_kcontig, b_kcontig, st);
    else if (kfull) e = gemm_launch_x3_t<true, false, 4>(g, grid, a_kcontig, b_kcontig, st);
    else e = gemm_launch_x3_t<false, false, 4>(g, grid, a_kcontig, b_kcontig, st);
  } else {
    if (kfull && pre) e = gemm_launch_x3_t<true, true, 2>(g, grid, a_kcontig, b_kcontig, st);
    else if (kfull) e = gemm_launch_x3_t<true, false, 2>(g, grid, a_kcontig, b_kcontig, st);
    else e = gemm_launch_x3_t<false, false, 2>(g, grid, a_kcontig, b_kcontig, st);
  }
  if (e) return e;
  return splitk_finish(a, split_k, slab_ws, st);
}

template <int BK, int BMT, int BNT>
int gemm_launch_t(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws, hipStream_t st) {
  lbwn_gemm_args g;
  dim3 grid;
  int e = gemm_setup(a, a_kcontig, b_kcontig, split_k, slab_ws, BK, BMT, BNT, g, grid);
  if (e) return e;
  if (a_kcontig && b_kcontig) gemm_f32_kernel<true, true, BK, BMT, BNT><<<grid, NT, 0, st>>>(g);
  else if (a_kcontig) gemm_f32_kernel<true, false, BK, BMT, BNT><<<grid, NT, 0, st>>>(g);
  else if (b_kcontig) gemm_f32_kernel<false, true, BK, BMT, BNT><<<grid, NT, 0, st>>>(g);
  else gemm_f32_kernel<false, false, BK, BMT, BNT><<<grid, NT, 0, st>>>(g);
  LBWN_CHECK_LAUNCH();
  return splitk_finish(a, split_k, slab_ws, st);
}
}  // namespace

// GEMM arithmetic: 1 = f32 operands split exactly into bf16 terms on the bf16 matrix cores
// (default), 0 = v_mfma_f32_32x32x2_f32.  LBWN_GEMM=f32 selects the latter at start-up.
static int g_gemm_mode = -1;
int lbwn_gemm_mode(void) {
  if (g_gemm_mode < 0) {
    const char* env = getenv("LBWN_GEMM");
    g_gemm_mode = (env && !strcmp(env, "f32")) ? 0 : 1;
  }
  return g_gemm_mode;
}
int lbwn_gemm_set_mode_impl(int mode) {
  LBWN_REQUIRE(mode == 0 || mode == 1, "gemm_set_mode: mode must be 0 (f32 MFMA) or 1 (bf16 split)");
  g_gemm_mode = mode;
  return 0;
}

bool lbwn_gemm_x3q8_form(int M, int N, int K, int a_kcontig, int presplit, int row_exact, int colpart) {
  const bool wm4 = colpart || (a_kcontig && N <= 2048 && (M >= 8192 || row_exact));
  return X3Q && lbwn_gemm_mode() == 1 && M >= 4 && N >= 4 && K >= 4 && wm4 && presplit && a_kcontig &&
         K % X3_BK == 0 && !(N <= 96) && !(N % 160 == 0 && N > 512);
}

int lbwn_gemm_launch(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws,
                     hipStream_t st) {
  if (lbwn_gemm_mode() == 1 && a.a_codes == nullptr && a.K >= 4 && a.M >= 4 && a.N >= 4)
    return gemm_launch_x3(a, a_kcontig, b_kcontig, split_k, slab_ws, st);
  LBWN_REQUIRE(a.colpart == nullptr && a.step_advance == nullptr && !a.c_chain_ls,
               "gemm: column partials / the step counter / chain-order C need the bf16-split form");
  return gemm_launch_t<16, 128, 128>(a, a_kcontig, b_kcontig, split_k, slab_ws, st);
}

int lbwn_gemm_launch_lean(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws,
                          hipStream_t st) {
  if (lbwn_gemm_mode() == 1 && a.a_codes == nullptr && a.K >= 4 && a.M >= 4 && a.N >= 4)
    return gemm_launch_x3(a, a_kcontig, b_kcontig, split_k, slab_ws, st);
  LBWN_REQUIRE(a.colpart == nullptr, "gemm: column partials need the bf16-split form");
  return gemm_launch_t<8, 128, 128>(a, a_kcontig, b_kcontig, split_k, slab_ws, st);
}

size_t lbwn_split_planes_elems(int rows, int K) { return (size_t)rows * ((K + X3_BK - 1) / X3_BK) * 3 * X3_BK; }

int lbwn_split_planes_launch(int njobs, const float* const* W, const long* ldw, const int* rows, const int* K,
                             const int* trans, unsigned short* const* out, hipStream_t st) {
  LBWN_REQUIRE(njobs >= 1 && njobs <= 6, "split_planes: 1..6 jobs");
  SplitJobs jb;
  memset(&jb, 0, sizeof(jb));
  long most = 0;
  for (int j = 0; j < njobs; ++j) {
    LBWN_REQUIRE(W[j] && out[j] && rows[j] > 0 && K[j] > 0, "split_planes: bad arguments");
    jb.W[j] = W[j]; jb.ldw[j] = ldw[j]; jb.rows[j] = rows[j]; jb.K[j] = K[j]; jb.trans[j] = trans[j]; jb.out[j] = out[j];
    most = std::max(most, (long)rows[j] * ((K[j] + X3_BK - 1) / X3_BK) * (X3_BK / 2));
  }
  const int blocks = (int)std::min<long>((most + 255) / 256, 1024);
  split_planes_kernel<<<dim3(blocks, njobs), 256, 0, st>>>(jb);
  LBWN_CHECK_LAUNCH();
  return 0;
}
