// Byte-/bandwidth-bound kernels around the residual stack:
//   D-separation prepend/save (tmodel.py:122-127, :165), PRE embedding (tmodel.py:53-66,
//   :86-102), the softmax-xent head with the invalid-window mask (tmodel.py:218-289),
//   column sums for bias grads, TF1 Adam (train.py:178, :186) and the µ-law codec
//   (ops.py:4-39).
#include <cstdio>
#include <math.h>

#include <string.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prologue.h"

namespace {

// ---- D-separation state and embedding: bodies in prologue.h ---------------------------------
template <bool TO_X>
__global__ void dsep_kernel(float* xall, long xls, float* save, int L, int nbl, int B, int T, int H, int Cr, bool v4) {
  dsep_flat_body<TO_X>(blockIdx.x, gridDim.x, xall, xls, save, L, nbl, B, T, H, Cr, v4);
}

__global__ void embed_kernel(const int* __restrict__ q, const float* __restrict__ pre, const float* pre_b,
                             float* x0, int B, int T, int H, int Cr, int Q, bool v4) {
  embed_flat_body(blockIdx.x, gridDim.x, q, pre, pre_b, x0, B, T, H, Cr, Q, v4);
}

// out[m] = a[m] + (t+gd < T ? c0[m+gd] : 0)   (dx of a layer input from (g + dcur, dprev))
__global__ void shift_add_kernel(float* out, const float* a, const float* c0, int gd, int B, int T, int C) {
  const long n = (long)B * T * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long m = e / C;
    const int t = (int)(m % T);
    float v = a[e];
    if (t + gd < T) v += c0[e + (long)gd * C];
    out[e] = v;
  }
}

// ---- PRE-embedding gradient -------------------------------------------------------------
// dPRE[q][c] = Σ_{t: code_t = q} dx0[t][c] and dPRE_B[c] = Σ_t dx0[t][c]: the transpose of the
// one-hot product (tmodel.py:64-66; tf.one_hot: a code outside [0, Q) has no row).  A scatter
// into an LDS histogram, not a dense GEMM against the one-hot matrix (K = B·T, M = Q, N = Cr:
// ~200 µs of tiles that are almost all zeros).  dx0 = g + shift(dprev) (layer 0's input
// gradient, as shift_add forms it) is formed on the fly and never stored.  Each wave of a block
// owns an LDS histogram and a contiguous sub-chunk of the block's positions, walked two positions
// per instruction (half-wave h takes h, h+2, ...) with no-return LDS float atomics (ds_add_f32:
// no read-modify-write round trip); a single wave's atomics are applied in program and lane
// order, the block's wave histograms are summed in wave order and the block partials are reduced
// in a fixed order, so the sums are deterministic.  Default 256 one-wave blocks (32 KB of LDS
// each, so they find room beside dSKIP's GEMM blocks; 128 x 1 and 256 x 2 measured slower).
constexpr int PG_BLOCKS = 256;
constexpr int PG_WAVES = 2;
constexpr int PG_BATCH = 4;    // small: <= 32 VGPRs so the blocks fit beside dSKIP's (see below)

// At most 32 VGPRs (27 / 25 for the reduce at this writing): it runs beside dSKIP's A-in-registers GEMM (2 waves of 240 VGPRs per SIMD)
__global__ __launch_bounds__(64 * PG_WAVES) void pre_grad_part_kernel(
    const int* __restrict__ q,
                                                                      const float* __restrict__ g,
                                                                      const float* __restrict__ dprev, int gd, int B,
                                                                      int T, int Cr, int Q, float* part, float* bpart) {
  extern __shared__ __attribute__((aligned(16))) float hist_all[];   // [nw][Q][32]
  __shared__ float bred[PG_WAVES][32];
  const int nw = blockDim.x >> 6;   // PG_WAVES, or 1 when two histograms exceed 64 KB (Q > 256)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = lane >> 5, c = lane & 31, cc = min(c, Cr - 1);
  float* hist = hist_all + (long)wv * Q * 32;
  for (int i = threadIdx.x; i < nw * Q * 32 / 4; i += 64 * nw)
    ((float4*)hist_all)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const long M = (long)B * T;
  const long chunk = (M + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * chunk, b1 = min(M, b0 + chunk);
  const long sub = (chunk + nw - 1) / nw, m0 = b0 + wv * sub, m1 = min(b1, m0 + sub);
  float bsum = 0.f;
  // 32-bit position arithmetic (M·Cr < 2^31, checked by the launcher): the kernel must stay within
  // the 32 VGPRs dSKIP's blocks leave per SIMD
  const int Mi = (int)M, m1i = (int)m1;
  for (int mb = (int)m0 + h; mb < m1i; mb += 2 * PG_BATCH) {
    int cd[PG_BATCH];
    float v[PG_BATCH], w[PG_BATCH];
#pragma unroll
    for (int i = 0; i < PG_BATCH; ++i) {   // loads first (clamped indices: no branch per load)
      const int m = min(mb + 2 * i, m1i - 1);
      const int ms = min(m + gd, Mi - 1);
      cd[i] = q[m];
      v[i] = g[m * Cr + cc];
      w[i] = dprev[ms * Cr + cc];
    }
#pragma unroll
    for (int i = 0; i < PG_BATCH; ++i) {
      const int m = mb + 2 * i;
      if (m >= m1i || c >= Cr) continue;
      const float x = v[i] + (m % T + gd < T ? w[i] : 0.f);
      bsum += x;
      if (cd[i] >= 0 && cd[i] < Q)
        __hip_atomic_fetch_add(hist + cd[i] * 32 + c, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  const float bo = __shfl_xor(bsum, 32);
  if (lane < 32) bred[wv][lane] = bsum + bo;
  __syncthreads();
  float* P = part + (long)blockIdx.x * Q * Cr;
  for (int e = threadIdx.x; e < Q * Cr; e += 64 * nw) {
    const int qq = e / Cr, c2 = e % Cr;
    float s = hist_all[qq * 32 + c2];
    for (int k = 1; k < nw; ++k) s += hist_all[(long)k * Q * 32 + qq * 32 + c2];
    P[e] = s;
  }
  if (threadIdx.x < Cr) {
    float s = bred[0][threadIdx.x];
    for (int k = 1; k < nw; ++k) s += bred[k][threadIdx.x];
    bpart[(long)blockIdx.x * Cr + threadIdx.x] = s;
  }
}

// 256 threads = 16 part lanes x 16 columns per block: lane pl sums partials pl, pl + 16, ... in
// order, then the 16 lane sums are added in order (deterministic).  (One thread per column
// walking all 256 partials ran 50 us beside dSKIP.)
__global__ __launch_bounds__(256) void pre_grad_reduce_kernel(
    const float* part, const float* bpart, int nparts,
                                                              int Q, int Cr, float* dpre, float* dpre_b) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int e = blockIdx.x * 16 + cl, n = Q * Cr;
  const bool bias = e >= n;
  const bool live = bias ? (dpre_b != nullptr && e - n < Cr) : true;
  const float* p = bias ? bpart + min(e - n, Cr - 1) : part + e;
  const long stride = bias ? Cr : n;
  float s = 0.f;
  if (live) {
    const int sti = (int)stride;
    for (int q0 = pl; q0 < nparts; q0 += 64) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = p[min(q0 + 16 * i, nparts - 1) * sti];
#pragma unroll
      for (int i = 0; i < 4; ++i) s += (q0 + 16 * i < nparts) ? v[i] : 0.f;
    }
  }
  red[pl][cl] = s;
  __syncthreads();
  if (threadIdx.x < 16 && live) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    if (bias) dpre_b[e - n] = t;
    else dpre[e] = t;
  }
}

// ---- softmax cross-entropy head ------------------------------------------------------------
// One wave per position row; dlogits (unnormalised) written in place.

// wave-wide max / min / sum on DPP (quad xor 1, 2, row_half_mirror, row_mirror: every row of 16
// uniform) and the four row values by readlane: one VALU latency per step instead of a ds_bpermute
// round trip per __shfl step (head_reg_kernel: 23.6 -> 21.3 us at C2, same box).  The sum order is
// fixed: quads, pairs of quads, half rows, then rows 0 + 1 + 2 + 3.
template <int CTRL>
LBWN_DEV int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
template <int CTRL>
LBWN_DEV float dpp_f(float v) { return __int_as_float(dpp_i<CTRL>(__float_as_int(v))); }
LBWN_DEV float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
LBWN_DEV int wave_min(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x141>(v));
  v = min(v, dpp_i<0x140>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
LBWN_DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return ((r0 + r1) + r2) + r3;
}

__global__ __launch_bounds__(256) void head_kernel(lbwn_head_args a) {
  __shared__ float part[4][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long M = (long)a.B * a.T;
  float s_xent = 0.f, s_valid = 0.f, s_diff = 0.f;
  for (long m = (long)blockIdx.x * 4 + w; m < M; m += (long)gridDim.x * 4) {
    float* row = a.logits + m * a.Q;
    const int t = (int)(m % a.T);
    if (t == a.T - 1) {  // logits_out[:, :-1] (tmodel.py:231): the last position has no target
      if (a.write_grad)
        for (int c = lane; c < a.Q; c += 64) row[c] = 0.f;
      continue;
    }
    const int tgt = a.q[m + 1];
    const bool valid = a.ids[m + 1] != 0;   // tmodel.py:232
    // max + first argmax
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int c = lane; c < a.Q; c += 64) {
      const float v = row[c];
      if (v > mx) { mx = v; am = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o);
      const int oa = __shfl_xor(am, o);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    float se = 0.f;
    for (int c = lane; c < a.Q; c += 64) se += expf(row[c] - mx);
    se = wave_sum(se);
    const float lse = mx + logf(se);
    const float xent = lse - row[tgt];
    if (a.write_grad) {
      const float inv = 1.f / se;
      for (int c = lane; c < a.Q; c += 64) {
        float g = expf(row[c] - mx) * inv - (c == tgt ? 1.f : 0.f);
        row[c] = valid ? g : 0.f;
      }
    }
    if (lane == 0 && valid) {
      s_xent += xent;
      s_valid += 1.f;
      s_diff += fabsf((float)(tgt - am));
    }
  }
  if (lane == 0) {
    part[w][0] = s_xent;
    part[w][1] = s_valid;
    part[w][2] = s_diff;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    a.partial[blockIdx.x * 3 + k] = ((part[0][k] + part[1][k]) + part[2][k]) + part[3][k];
  }
}

// The same head with the row held in registers (Q <= 64·QV): one coalesced load pass, exp once,
// the gradient written from registers (the generic kernel above re-reads the row three times and
// evaluates exp twice).  Lane c-order (c = lane + 64·j) and the first-max tie-break are kept, so
// argmax (avg_diff) is identical; Σe is summed per lane, then across the wave.
// With a.colpart, the block's column sums of the dlogits it wrote go to colpart[block][Q] (the
// post2 bias gradient's partials, summed by colsum_final: no second pass over the [M][Q] matrix).
template <int QV>
__global__ __launch_bounds__(256) void head_reg_kernel(lbwn_head_args a) {
  __shared__ float part[4][3];
  __shared__ float cpart[4][64 * QV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long M = (long)a.B * a.T;
  const int Q = a.Q;
  float s_xent = 0.f, s_valid = 0.f, s_diff = 0.f;
  float cs[QV];
#pragma unroll
  for (int j = 0; j < QV; ++j) cs[j] = 0.f;
  // the next row's logits and target are loaded while this row is processed (one row of HBM
  // latency in flight per wave instead of none)
  const long stride = (long)gridDim.x * 4;
  long m = (long)blockIdx.x * 4 + w;
  float vn[QV];
  int tn = 0, idn = 0;
  {
    const long mc = min(m, M - 1), mq = min(mc + 1, M - 1);
#pragma unroll
    for (int j = 0; j < QV; ++j) vn[j] = a.logits[mc * Q + min(lane + 64 * j, Q - 1)];
    tn = a.q[mq];
    idn = a.ids[mq];
  }
  for (; m < M; m += stride) {
    float* row = a.logits + m * Q;
    float v[QV];
#pragma unroll
    for (int j = 0; j < QV; ++j) v[j] = (lane + 64 * j < Q) ? vn[j] : -INFINITY;
    const int tgt = tn;
    const bool valid = idn != 0;   // tmodel.py:232
    {
      const long mc = min(m + stride, M - 1), mq = min(mc + 1, M - 1);
#pragma unroll
      for (int j = 0; j < QV; ++j) vn[j] = a.logits[mc * Q + min(lane + 64 * j, Q - 1)];
      tn = a.q[mq];
      idn = a.ids[mq];
    }
    const int t = (int)(m % a.T);
    if (t == a.T - 1) {  // logits_out[:, :-1] (tmodel.py:231): the last position has no target
      if (a.write_grad)
#pragma unroll
        for (int j = 0; j < QV; ++j)
          if (lane + 64 * j < Q) row[lane + 64 * j] = 0.f;
      continue;
    }
    // max, then the first code holding it (the same first-max tie-break as a (value, index)
    // reduction, in two DPP passes)
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < QV; ++j) mx = fmaxf(mx, v[j]);
    mx = wave_max(mx);
    int am = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < QV; ++j)
      if (am == 0x7fffffff && v[j] == mx) am = lane + 64 * j;
    am = wave_min(am);
    float e[QV], se = 0.f, pick = 0.f;
#pragma unroll
    for (int j = 0; j < QV; ++j) {
      e[j] = (lane + 64 * j < Q) ? expf(v[j] - mx) : 0.f;
      se += e[j];
      if (lane + 64 * j == tgt) pick = v[j];
    }
    se = wave_sum(se);
    pick = wave_sum(pick);   // the one lane holding the target's logit; the rest add 0
    const float xent = (mx + logf(se)) - pick;
    if (a.write_grad) {
      const float inv = 1.f / se;
#pragma unroll
      for (int j = 0; j < QV; ++j) {
        const int c = lane + 64 * j;
        const float g = valid ? e[j] * inv - (c == tgt ? 1.f : 0.f) : 0.f;
        if (c < Q) row[c] = g;
        cs[j] += g;
      }
    }
    if (lane == 0 && valid) {
      s_xent += xent;
      s_valid += 1.f;
      s_diff += fabsf((float)(tgt - am));
    }
  }
  if (lane == 0) {
    part[w][0] = s_xent;
    part[w][1] = s_valid;
    part[w][2] = s_diff;
  }
  if (a.colpart) {
#pragma unroll
    for (int j = 0; j < QV; ++j) cpart[w][lane + 64 * j] = cs[j];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    a.partial[blockIdx.x * 3 + k] = ((part[0][k] + part[1][k]) + part[2][k]) + part[3][k];
  }
  if (a.colpart)
    for (int c = threadIdx.x; c < Q; c += 256)
      a.colpart[(long)blockIdx.x * Q + c] = ((cpart[0][c] + cpart[1][c]) + cpart[2][c]) + cpart[3][c];
}

// stats[0] = Σxent, [1] = n_valid, [2] = Σ|diff|, [3] = 1/n_valid (0 if none)
__global__ void stats_reduce_kernel(const float* partial, int nparts, float* stats) {
  __shared__ double sh[3][256];
  double s[3] = {0, 0, 0};
  for (int p = threadIdx.x; p < nparts; p += blockDim.x)
    for (int k = 0; k < 3; ++k) s[k] += partial[p * 3 + k];
  for (int k = 0; k < 3; ++k) sh[k][threadIdx.x] = s[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int k = 0; k < 3; ++k) sh[k][threadIdx.x] += sh[k][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[0] = (float)sh[0][0];
    stats[1] = (float)sh[1][0];
    stats[2] = (float)sh[2][0];
    stats[3] = sh[1][0] > 0 ? (float)(1.0 / sh[1][0]) : 0.f;
  }
}

// ---- column sums (bias gradients), deterministic two-pass ------------------------------------
// pass 1: block = CS_ROWS rows × all N columns (float4 groups × row lanes); pass 2: 1024
// threads per 64 columns sum the chunk partials.  N % 4 == 0, N <= 1024.

constexpr int CS_ROWS = 64;
// up to 4 column sums of M-row matrices in one launch pair (blockIdx.y = job)
struct ColsumJobs {
  const float* X[4];
  long ldx[4];
  int N[4];
  float* out[4];
  int accumulate[4];
  float* ws[4];
  int nparts[4];   // partial rows per job (colsum_final_kernel)
  int reps[4];     // copies of the result row written (out + r·N), colsum_final_kernel
};
__global__ __launch_bounds__(256) void colsum_partial_kernel(ColsumJobs jb, int M) {
  __shared__ floatx4 red[256];
  const int j = blockIdx.y;
  const float* X = jb.X[j];
  const long ldx = jb.ldx[j];
  const int N = jb.N[j];
  float* part = jb.ws[j];
  const int ng = N / 4, RL = max(1, 256 / ng);
  const int t = threadIdx.x, g = t % ng, rl = t / ng;
  const int r0 = blockIdx.x * CS_ROWS;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  if (rl < RL && g < ng) {
    const int r1 = min(M, r0 + CS_ROWS);
#pragma unroll 8
    for (int r = r0 + rl; r < r1; r += RL) s += *(const floatx4*)(X + (long)r * ldx + 4 * g);
  }
  red[t] = s;
  __syncthreads();
  if (t < ng) {
    floatx4 tot = red[t];
    for (int k = 1; k < RL; ++k) tot += red[k * ng + t];
    *(floatx4*)(part + (long)blockIdx.x * N + 4 * t) = tot;
  }
}
// 256 threads = 16 part lanes × 16 columns per block (grid: N/16 column blocks × jobs): each lane
// sums every 16th partial row in order, then the 16 lane sums are added in order (deterministic).
// (4 part lanes × 64 columns left 256-deep serial sums per thread once the head wrote 1024
// partial rows: 21 µs for the three bias sums)
__global__ __launch_bounds__(256) void colsum_final_kernel(ColsumJobs jb) {
  __shared__ float red[16][17];
  const int j = blockIdx.y, N = jb.N[j], nparts = jb.nparts[j];
  const float* part = jb.ws[j];
  const int cl = threadIdx.x & 15, lane = threadIdx.x >> 4, c = blockIdx.x * 16 + cl;
  if (blockIdx.x * 16 >= N) return;   // block-uniform
  float s = 0.f;
  if (c < N) {
#pragma unroll 8
    for (int p = lane; p < nparts; p += 16) s += part[(long)p * N + c];
  }
  red[lane][cl] = s;
  __syncthreads();
  if (threadIdx.x < 16 && c < N) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) tot += red[k][cl];
    float* out = jb.out[j];
    for (int r = 0; r < max(1, jb.reps[j]); ++r) {
      float* o = out + (long)r * N + c;
      *o = jb.accumulate[j] ? *o + tot : tot;
    }
  }
}

__global__ void sum_bias_kernel(const float* b, int L, int N, float* out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
#pragma unroll 10
  for (int l = 0; l < L; ++l) s += b[(long)l * N + n];
  out[n] = s;
}

__global__ void fill_kernel(float* p, float v, long n) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) p[e] = v;
}

// ---- TF1 Adam over the flat parameter buffer --------------------------------------------------
// grads hold Σ-xent gradients; g = raw·(1/n_valid) + l2·θ for the weight region
// [0, n_weights) (non-BIAS vars, tmodel.py:250-261); biases get no l2 term.
// counters[2] (int64) is Adam's apply count t-1; lr_t = lr·√(1-β2^t)/(1-β1^t).
// status (nullable): the step's chain status word; nonzero = a hand-off timed out and the
// gradients are garbage, so the update is skipped (params, m, v untouched).
// one element of TF1 Adam (training_ops.cc ApplyAdam restated: m, v, then θ -= lr_t·m/(√v + ε))
LBWN_DEV float adam_elem(float th, float g, float& m, float& v, float lr_t, float b1, float b2, float eps) {
  const float mm = b1 * m + (1.f - b1) * g;
  const float vv = b2 * v + (1.f - b2) * g * g;
  m = mm;
  v = vv;
  return th - lr_t * mm / (sqrtf(vv) + eps);
}

// Four elements per thread as dwordx4 loads and stores (the flat buffers are 16-B aligned, checked
// by the launcher); the n % 4 tail elements one per thread.  HBM-bound: 28 B per parameter.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ gr,
                                                   float* __restrict__ m, float* __restrict__ v, long nw, long n,
                                                   float lr, float b1, float b2, float eps, float l2,
                                                   const float* stats, const long long* counters,
                                                   const unsigned* status) {
  if (status && *status) return;
  const double t = (double)(counters[2] + 1);
  const float lr_t = (float)((double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t)));
  const float inv = stats ? (stats[1] > 0.f ? 1.f / stats[1] : 0.f) : 1.f;
  const long n4 = n >> 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const floatx4 th = ((const floatx4*)p)[i];
    floatx4 g = ((const floatx4*)gr)[i];
    floatx4 mm = ((const floatx4*)m)[i], vv = ((const floatx4*)v)[i], out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * inv;
      if (4 * i + j < nw) gj += l2 * th[j];
      float mj = mm[j], vj = vv[j];
      out[j] = adam_elem(th[j], gj, mj, vj, lr_t, b1, b2, eps);
      mm[j] = mj;
      vv[j] = vj;
    }
    ((floatx4*)m)[i] = mm;
    ((floatx4*)v)[i] = vv;
    ((floatx4*)p)[i] = out;
  }
  const long e = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e < n) {
    float g = gr[e] * inv;
    if (e < nw) g += l2 * p[e];
    float mj = m[e], vj = v[e];
    p[e] = adam_elem(p[e], g, mj, vj, lr_t, b1, b2, eps);
    m[e] = mj;
    v[e] = vj;
  }
}

// counters: [0] GLOBAL_STEP, [1] VALID_SAMPLES, [2] Adam t-1 (tmodel.py:282-287), [3] the
// cumulative status: every step's status word ORed in (never reset by a step), so one read
// after many steps tells whether any of them timed out.  A failed step advances nothing else.
__global__ void counters_kernel(long long* counters, const float* stats, int adam_applied, const unsigned* status) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const unsigned s = status ? *status : 0u;
    if (s) {
      counters[3] |= (long long)s;
      return;
    }
    counters[0] += 1;
    counters[1] += (long long)stats[1];
    counters[2] += adam_applied;
  }
}

// ---- µ-law ---------------------------------------------------------------------------------

__global__ void mulaw_encode_kernel(const float* x, int* q, long n, int nq, int tf32) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    if (tf32) {  // ops.py:4-9, float32 throughout
      const float mu = (float)(nq - 1), xv = x[e];
      const float sg = xv > 0.f ? 1.f : (xv < 0.f ? -1.f : 0.f);
      const float amp = sg * log1pf(mu * fabsf(xv)) / log1pf(mu);
      q[e] = (int)((amp + 1.f) * 0.5f * mu + 0.5f);
    } else {  // ops.py:23-28, numpy float64
      const double mu = (double)(nq - 1), xv = (double)x[e];
      const double sg = xv > 0 ? 1.0 : (xv < 0 ? -1.0 : 0.0);
      const double amp = sg * log1p(mu * fabs(xv)) / log1p(mu);
      q[e] = (int)((amp + 1.0) * 0.5 * mu + 0.5);
    }
  }
}

__global__ void mulaw_decode_kernel(const int* q, float* x, long n, int nq) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const float mu = (float)(nq - 1), inv_mu = 1.f / mu;  // ops.py:12-20
    const float a = (2.f * (float)q[e] - 1.f) * inv_mu - 1.f;
    const float sg = a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f);
    x[e] = sg * (powf(1.f + mu, fabsf(a)) - 1.f) * inv_mu;
  }
}

inline int grid_for(long n, int per = 256, int cap = 8192) {
  long g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

}  // namespace

// one flat launch over every layer's SAVE rows (dsep_flat_body), one item per thread
static int dsep_launch(bool to_x, float* xall, long xls, float* save, int L, int nbl, int B, int T, int H, int Cr,
                       hipStream_t st) {
  LBWN_REQUIRE(L >= 1 && nbl >= 1 && nbl <= 16 && B >= 1 && Cr >= 1, "dsep: bad shape");
  LBWN_REQUIRE((long)dsep_rows(L, nbl, 1) * B * Cr < (1L << 31), "dsep: SAVE exceeds 32-bit indexing");
  const bool v4 = dsep_v4(xall, xls, save, Cr);
  const long n = (long)dsep_rows(L, nbl, B) * (v4 ? Cr / 4 : Cr);
  const int grid = (int)std::max(1L, std::min(2048L, (n + 255) / 256));
  if (to_x) dsep_kernel<true><<<grid, 256, 0, st>>>(xall, xls, save, L, nbl, B, T, H, Cr, v4);
  else dsep_kernel<false><<<grid, 256, 0, st>>>(xall, xls, save, L, nbl, B, T, H, Cr, v4);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_dsep_prepend_launch(float* xall, long xls, const float* save, int L, int nbl, int B, int T, int H,
                             int Cr, hipStream_t st) {
  return dsep_launch(true, xall, xls, const_cast<float*>(save), L, nbl, B, T, H, Cr, st);
}

int lbwn_dsep_save_launch(const float* xall, long xls, float* save, int L, int nbl, int B, int T, int H, int Cr,
                          hipStream_t st) {
  return dsep_launch(false, const_cast<float*>(xall), xls, save, L, nbl, B, T, H, Cr, st);
}

int lbwn_embed_launch(const int* q, const float* pre, const float* pre_b, float* x0, int B, int T, int H, int Cr,
                      int Q, hipStream_t st) {
  LBWN_REQUIRE((long)B * T * Cr < (1L << 31), "embed: B*T*n_res exceeds 32-bit indexing");
  const bool v4 = embed_v4(pre, pre_b, x0, Cr);
  embed_kernel<<<grid_for((long)B * T * (v4 ? Cr / 4 : Cr)), 256, 0, st>>>(q, pre, pre_b, x0, B, T, H, Cr, Q, v4);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_pre_grad_ws_floats(int Q, int Cr) { return PG_BLOCKS * (Q * Cr + Cr); }

int lbwn_pre_grad_launch(const int* q, const float* g, const float* dprev, int gd, int B, int T, int Cr, int Q,
                         float* dpre, float* dpre_b, float* ws, hipStream_t st) {
  LBWN_REQUIRE(Cr >= 1 && Cr <= 32 && Q >= 1 && Q * 32 * 4 <= 65536, "pre_grad: Cr <= 32 and Q <= 512 required");
  LBWN_REQUIRE((long)B * T * Cr < (1L << 31), "pre_grad: B*T*Cr must be < 2^31");
  const int nb = PG_BLOCKS, nw = 1;   // one-wave blocks (two-wave blocks wait for LDS)
  float* part = ws;
  float* bpart = ws + (long)PG_BLOCKS * Q * Cr;
  pre_grad_part_kernel<<<nb, 64 * nw, nw * Q * 32 * 4, st>>>(q, g, dprev, gd, B, T, Cr, Q, part, bpart);
  LBWN_CHECK_LAUNCH();
  const int n = Q * Cr + Cr;
  pre_grad_reduce_kernel<<<(n + 15) / 16, 256, 0, st>>>(part, bpart, nb, Q, Cr, dpre, dpre_b);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_shift_add_launch(float* out, const float* a, const float* c0, int gd, int B, int T, int C,
                          hipStream_t st) {
  shift_add_kernel<<<grid_for((long)B * T * C), 256, 0, st>>>(out, a, c0, gd, B, T, C);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_head_launch(const lbwn_head_args& a, int* nblocks_out, hipStream_t st) {
  const long M = (long)a.B * a.T;
  LBWN_REQUIRE(!a.colpart || a.Q <= 512, "head: column partials need Q <= 512");
  const int nb = lbwn_head_nblocks(M, a.colpart != nullptr);
  if (a.Q <= 256) head_reg_kernel<4><<<nb, 256, 0, st>>>(a);
  else if (a.Q <= 512) head_reg_kernel<8><<<nb, 256, 0, st>>>(a);
  else head_kernel<<<nb, 256, 0, st>>>(a);
  LBWN_CHECK_LAUNCH();
  if (nblocks_out) *nblocks_out = nb;
  return 0;
}
// with column partials: at most ceil(M/32) blocks, so colpart fits the colsum workspace
int lbwn_head_nblocks(long M, bool colpart) {
  return (int)(colpart ? std::min<long>((M + 31) / 32, 1024) : std::min<long>((M + 3) / 4, 2048));
}

int lbwn_stats_reduce_launch(const float* partial, int nparts, float* stats, hipStream_t st) {
  stats_reduce_kernel<<<1, 256, 0, st>>>(partial, nparts, stats);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_colsum_ws_floats(int M, int N) { return ((M + CS_ROWS - 1) / CS_ROWS) * N; }

int lbwn_colsum_multi_launch(int njobs, const float* const* X, const long* ldx, const int* N, float* const* out,
                             const int* accumulate, int M, float* ws, hipStream_t st) {
  LBWN_REQUIRE(njobs >= 1 && njobs <= 4, "colsum: 1..4 jobs");
  ColsumJobs jb;
  memset(&jb, 0, sizeof(jb));
  const int np = (M + CS_ROWS - 1) / CS_ROWS;
  int nmax = 0;
  float* w = ws;
  for (int j = 0; j < njobs; ++j) {
    LBWN_REQUIRE(N[j] % 4 == 0 && N[j] <= 1024 && ldx[j] % 4 == 0, "colsum: N %% 4 / N <= 1024 / ldx %% 4 required");
    jb.X[j] = X[j]; jb.ldx[j] = ldx[j]; jb.N[j] = N[j]; jb.out[j] = out[j]; jb.accumulate[j] = accumulate[j];
    jb.ws[j] = w;
    jb.nparts[j] = np;
    w += (long)np * N[j];
    nmax = std::max(nmax, N[j]);
  }
  colsum_partial_kernel<<<dim3(np, njobs), 256, 0, st>>>(jb, M);
  colsum_final_kernel<<<dim3((nmax + 15) / 16, njobs), 256, 0, st>>>(jb);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_colsum_partial_launch(const float* X, long ldx, int M, int N, float* ws, int* nparts, hipStream_t st) {
  LBWN_REQUIRE(N % 4 == 0 && N <= 1024 && ldx % 4 == 0, "colsum: N %% 4 / N <= 1024 / ldx %% 4 required");
  ColsumJobs jb;
  memset(&jb, 0, sizeof(jb));
  jb.X[0] = X; jb.ldx[0] = ldx; jb.N[0] = N; jb.ws[0] = ws;
  const int np = (M + CS_ROWS - 1) / CS_ROWS;
  colsum_partial_kernel<<<dim3(np, 1), 256, 0, st>>>(jb, M);
  LBWN_CHECK_LAUNCH();
  *nparts = np;
  return 0;
}

int lbwn_colsum_final_launch(int njobs, float* const* parts, const int* N, float* const* out, const int* accumulate,
                             const int* nparts, hipStream_t st, const int* reps) {
  LBWN_REQUIRE(njobs >= 1 && njobs <= 4, "colsum_final: 1..4 jobs");
  ColsumJobs jb;
  memset(&jb, 0, sizeof(jb));
  int nmax = 0;
  for (int j = 0; j < njobs; ++j) {
    LBWN_REQUIRE(nparts[j] >= 1, "colsum_final: nparts >= 1");
    jb.N[j] = N[j]; jb.out[j] = out[j]; jb.accumulate[j] = accumulate[j]; jb.ws[j] = parts[j];
    jb.nparts[j] = nparts[j];
    jb.reps[j] = reps ? reps[j] : 1;
    nmax = std::max(nmax, N[j]);
  }
  colsum_final_kernel<<<dim3((nmax + 15) / 16, njobs), 256, 0, st>>>(jb);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_colsum_launch(const float* X, long ldx, int M, int N, float* out, int accumulate, float* ws,
                       hipStream_t st) {
  return lbwn_colsum_multi_launch(1, &X, &ldx, &N, &out, &accumulate, M, ws, st);
}

int lbwn_sum_bias_launch(const float* b, int L, int N, float* out, hipStream_t st) {
  sum_bias_kernel<<<(N + 63) / 64, 64, 0, st>>>(b, L, N, out);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_fill_launch(float* p, float v, long n, hipStream_t st) {
  fill_kernel<<<grid_for(n), 256, 0, st>>>(p, v, n);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_adam_launch2(float* params, const float* grads, float* m, float* v, long nw, long n, float lr, float b1,
                      float b2, float eps, float l2, const float* stats, const long long* counters, const unsigned* status,
                      hipStream_t st) {
  LBWN_REQUIRE(!(((uintptr_t)params | (uintptr_t)grads | (uintptr_t)m | (uintptr_t)v) & 15),
               "adam: parameter, gradient and slot buffers must be 16-byte aligned");
  adam_kernel<<<grid_for(std::max(n / 4, 1L), 256, 4096), 256, 0, st>>>(params, grads, m, v, nw, n, lr, b1, b2, eps,
                                                                        l2, stats, counters, status);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_counters_launch(long long* counters, const float* stats, int adam_applied, const unsigned* status,
                         hipStream_t st) {
  counters_kernel<<<1, 64, 0, st>>>(counters, stats, adam_applied, status);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_mulaw_encode_launch(const float* x, int* q, long n, int nq, int tf32, hipStream_t st) {
  mulaw_encode_kernel<<<grid_for(n), 256, 0, st>>>(x, q, n, nq, tf32);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_mulaw_decode_launch(const int* q, float* x, long n, int nq, hipStream_t st) {
  mulaw_decode_kernel<<<grid_for(n), 256, 0, st>>>(q, x, n, nq);
  LBWN_CHECK_LAUNCH();
  return 0;
}

namespace {
__global__ void bcast_rows_kernel(float* dst, int L, int N) {
  // dst[l][n] = dst[0][n] for l in [1, L)
  const long n_all = (long)(L - 1) * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n_all; e += (long)gridDim.x * blockDim.x)
    dst[N + e] = dst[e % N];
}
}  // namespace

namespace {
__global__ void zero_words_kernel(unsigned* p, long n) { zero_body(blockIdx.x, gridDim.x, p, n); }
}  // namespace

// Zero n_bytes (a multiple of 4) on the stream: an ordinary kernel in the step's launch sequence.
// hipMemsetAsync's fill kernel started 13-18 us after the kernel before it (runtime blit path;
// profiles/r03_v2_step_timeline.txt: counters -> fill at the step start), a plain launch ~2 us.
int lbwn_zero_launch(void* p, size_t n_bytes, hipStream_t st) {
  LBWN_REQUIRE(n_bytes % 4 == 0, "zero: byte count must be a multiple of 4");
  const long n = (long)(n_bytes / 4);
  if (n == 0) return 0;
  zero_words_kernel<<<grid_for(n, 256, 1024), 256, 0, st>>>((unsigned*)p, n);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_bcast_rows_launch(float* dst, int L, int N, hipStream_t st) {
  if (L <= 1) return 0;
  bcast_rows_kernel<<<grid_for((long)(L - 1) * N), 256, 0, st>>>(dst, L, N);
  LBWN_CHECK_LAUNCH();
  return 0;
}
