// Global / local conditioning (tmodel.py:68-83, :92-114, :150-160).
//
// GC: the per-layer term GC_EMBED[ids]·GC_k_l depends on the position only through its
// voice id, so it is a lookup in a per-step table GCTAB[c][l][sig Cd | gate Cd] =
// GC_EMBED[c]·[GC_SIGNAL_l | GC_GATE_l]; the layer kernels add row ids[m].  Backward: the
// layer kernels scatter-add dv rows into GCD[c][l][2Cd] (per voice id), and
//   dGC_SIGNAL_l = GC_EMBEDᵀ·GCD_l[:, :Cd],  dGC_EMBED = Σ_l GCD_l·[GC_SIGNAL_l | GC_GATE_l]ᵀ.
// LC: the per-layer projections LC_SIGNAL_l / LC_GATE_l are packed side by side into one
// [Clc][L·2Cd] matrix so the whole conditioning input is ONE GEMM lc·LCcat (engine.cpp).
#include "common.h"
#include "kernels.h"

namespace {

// Tables are [ncat+1][L·2Cd]: row c holds every layer's (sig Cd | gate Cd) block, n = l·2Cd + s·Cd + o.
LBWN_DEV const float* gc_w(const float* wsig, const float* wgate, int n, int e, int Ge, int Cd) {
  const int l = n / (2 * Cd), s = (n / Cd) & 1, o = n % Cd;
  return (s == 0 ? wsig : wgate) + ((long)l * Ge + e) * Cd + o;
}

// out[c][n] = Σ_e emb[c][e] · W(n)[e]
__global__ void gc_table_kernel(const float* __restrict__ emb, const float* __restrict__ wsig,
                                const float* __restrict__ wgate, float* __restrict__ out, int N, int ncat1, int Ge,
                                int Cd) {
  const long total = (long)ncat1 * N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i % N), c = (int)(i / N);
    const float* e = emb + (long)c * Ge;
    float acc = 0.f;
    for (int k = 0; k < Ge; ++k) acc += e[k] * *gc_w(wsig, wgate, n, k, Ge, Cd);
    out[i] = acc;
  }
}

constexpr int GC_CSPLIT = 16;   // category chunks of the weight-gradient pass
constexpr int GC_EMAX = 32;     // n_gc_embed supported by the gradient kernels

// part[k][e][n] = Σ_{c in chunk k} emb[c][e] · gcd[c][n]   (grid: n blocks × GC_CSPLIT chunks)
__global__ __launch_bounds__(256) void gc_wgrad_part_kernel(const float* __restrict__ emb,
                                                            const float* __restrict__ gcd, float* __restrict__ part,
                                                            int N, int ncat1, int Ge) {
  const int n = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y;
  const int per = (ncat1 + GC_CSPLIT - 1) / GC_CSPLIT, c0 = k * per, c1 = min(ncat1, c0 + per);
  float acc[GC_EMAX];
#pragma unroll
  for (int e = 0; e < GC_EMAX; ++e) acc[e] = 0.f;
  if (n < N) {
    for (int c = c0; c < c1; ++c) {
      const float g = gcd[(long)c * N + n];
#pragma unroll
      for (int e = 0; e < GC_EMAX; ++e)
        if (e < Ge) acc[e] += emb[(long)c * Ge + e] * g;
    }
#pragma unroll
    for (int e = 0; e < GC_EMAX; ++e)
      if (e < Ge) part[((long)k * Ge + e) * N + n] = acc[e];
  }
}

// dW(n)[e] = Σ_k part[k][e][n]  (fixed order: deterministic)
__global__ void gc_wgrad_sum_kernel(const float* __restrict__ part, float* __restrict__ dsig, float* __restrict__ dgate,
                                    int N, int Ge, int Cd) {
  const long total = (long)Ge * N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i % N), e = (int)(i / N);
    float s = 0.f;
    for (int k = 0; k < GC_CSPLIT; ++k) s += part[((long)k * Ge + e) * N + n];
    *const_cast<float*>(gc_w(dsig, dgate, n, e, Ge, Cd)) = s;
  }
}

// dEMB[c][e] = Σ_n gcd[c][n] · W(n)[e]: one block per category, wave-then-block reduction.
__global__ __launch_bounds__(256) void gc_egrad_kernel(const float* __restrict__ gcd, const float* __restrict__ wsig,
                                                       const float* __restrict__ wgate, float* __restrict__ demb,
                                                       int N, int Ge, int Cd) {
  __shared__ float red[4][GC_EMAX];
  const int c = blockIdx.x;
  float acc[GC_EMAX];
#pragma unroll
  for (int e = 0; e < GC_EMAX; ++e) acc[e] = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) {
    const float g = gcd[(long)c * N + n];
    const int l = n / (2 * Cd), s = (n / Cd) & 1, o = n % Cd;
    const float* W = (s == 0 ? wsig : wgate) + (long)l * Ge * Cd + o;
#pragma unroll
    for (int e = 0; e < GC_EMAX; ++e)
      if (e < Ge) acc[e] += g * W[(long)e * Cd];
  }
#pragma unroll
  for (int e = 0; e < GC_EMAX; ++e) {
    float v = acc[e];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    acc[e] = v;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < GC_EMAX; ++e) red[w][e] = acc[e];
  }
  __syncthreads();
  if ((int)threadIdx.x < Ge) demb[(long)c * Ge + threadIdx.x] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// LCcat[i][l·2Cd + s·Cd + o] = W_s[l][i][o]  (pack = 1)  or the inverse scatter (pack = 0)
__global__ void lc_pack_kernel(float* __restrict__ cat, float* __restrict__ wsig, float* __restrict__ wgate, int L,
                               int Clc, int Cd, int pack) {
  const long total = (long)Clc * L * 2 * Cd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i % ((long)L * 2 * Cd)), k = (int)(i / ((long)L * 2 * Cd));
    const int l = n / (2 * Cd), s = (n / Cd) & 1, o = n % Cd;
    float* w = (s == 0 ? wsig : wgate) + ((long)l * Clc + k) * Cd + o;
    if (pack) cat[i] = *w;
    else *w = cat[i];
  }
}

int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 4096); }

}  // namespace

int lbwn_gc_part_floats(int L, int Ge, int Cd) { return GC_CSPLIT * Ge * 2 * L * Cd; }

int lbwn_gc_table_launch(const float* emb, const float* wsig, const float* wgate, float* out, int L, int ncat1,
                         int Ge, int Cd, hipStream_t st) {
  const int N = 2 * L * Cd;
  gc_table_kernel<<<grid_for((long)ncat1 * N), 256, 0, st>>>(emb, wsig, wgate, out, N, ncat1, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_gc_grad_launch(const float* emb, const float* wsig, const float* wgate, const float* gcd, float* part,
                        float* demb, float* dsig, float* dgate, int L, int ncat1, int Ge, int Cd, hipStream_t st) {
  LBWN_REQUIRE(Ge >= 1 && Ge <= GC_EMAX, "gc grads: n_gc_embed must be in [1, %d]", GC_EMAX);
  const int N = 2 * L * Cd;
  gc_wgrad_part_kernel<<<dim3((N + 255) / 256, GC_CSPLIT), 256, 0, st>>>(emb, gcd, part, N, ncat1, Ge);
  LBWN_CHECK_LAUNCH();
  gc_wgrad_sum_kernel<<<grid_for((long)Ge * N), 256, 0, st>>>(part, dsig, dgate, N, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  gc_egrad_kernel<<<ncat1, 256, 0, st>>>(gcd, wsig, wgate, demb, N, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_lc_pack_launch(float* cat, float* wsig, float* wgate, int L, int Clc, int Cd, int pack, hipStream_t st) {
  lc_pack_kernel<<<grid_for((long)Clc * L * 2 * Cd), 256, 0, st>>>(cat, wsig, wgate, L, Clc, Cd, pack);
  LBWN_CHECK_LAUNCH();
  return 0;
}
