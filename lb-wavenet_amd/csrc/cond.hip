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

// dEMB[c][e] = Σ_n gcd[c][n] · W(n)[e] as a small tiled product: block (category group cg, n chunk
// k) stages gcd[cg·CPB .. +CPB][k·256 .. +256] and W(n)[0..Ge) for its 256 n into LDS with all
// loads issued at once, then thread (category cl, column e) sums its 256 products; the chunk
// partials part[k][c][e] are summed in chunk order by gc_egrad_sum_kernel (deterministic).
// (One block per category looping over n ran 114-308 µs: dependent load chains behind integer
// divisions; this form is one wave of ~300 blocks.)
constexpr int GE_N = 256;
__global__ __launch_bounds__(256) void gc_egrad_part_kernel(const float* __restrict__ gcd,
                                                            const float* __restrict__ wsig,
                                                            const float* __restrict__ wgate,
                                                            float* __restrict__ part, int N, int ncat1, int Ge,
                                                            int Cd) {
  __shared__ float gs[16][GE_N + 1];
  __shared__ float wsm[GE_N][GC_EMAX + 1];
  const int ep = Ge <= 16 ? 16 : 32, cpb = 256 / ep;
  const int cg = blockIdx.x, k = blockIdx.y, t = threadIdx.x;
  const int n = k * GE_N + t, nc = min(n, N - 1);
  {
    const int l = nc / (2 * Cd), s = (nc / Cd) & 1, o = nc % Cd;
    const float* W = (s == 0 ? wsig : wgate) + (long)l * Ge * Cd + o;
    float wv[GC_EMAX], gv[16];
#pragma unroll
    for (int e = 0; e < GC_EMAX; ++e) wv[e] = W[(long)min(e, Ge - 1) * Cd];
#pragma unroll
    for (int c = 0; c < 16; ++c) gv[c] = gcd[(long)min(cg * cpb + min(c, cpb - 1), ncat1 - 1) * N + nc];
    const bool in = n < N;
#pragma unroll
    for (int e = 0; e < GC_EMAX; ++e) wsm[t][e] = in ? wv[e] : 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) gs[c][t] = in ? gv[c] : 0.f;
  }
  __syncthreads();
  const int cl = t / ep, e = t % ep, c = cg * cpb + cl;
  float acc = 0.f;
#pragma unroll 8
  for (int j = 0; j < GE_N; ++j) acc += gs[cl][j] * wsm[j][e];
  if (c < ncat1 && e < Ge) part[((long)k * ncat1 + c) * Ge + e] = acc;
}

__global__ void gc_egrad_sum_kernel(const float* __restrict__ part, float* __restrict__ demb, int nk, int ncat1,
                                    int Ge) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncat1 * Ge) return;
  float s = 0.f;
  for (int k = 0; k < nk; ++k) s += part[(long)k * ncat1 * Ge + i];
  demb[i] = s;
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
  // (part is free again: gc_wgrad_sum_kernel consumed it; GC_CSPLIT·Ge·N >= nk·ncat1·Ge floats
  // holds for every shipped arch and is checked here)
  const int nk = (N + GE_N - 1) / GE_N, ep = Ge <= 16 ? 16 : 32, cpb = 256 / ep;
  LBWN_REQUIRE((long)nk * ncat1 * Ge <= (long)GC_CSPLIT * Ge * N, "gc grads: partial buffer too small");
  gc_egrad_part_kernel<<<dim3((ncat1 + cpb - 1) / cpb, nk), 256, 0, st>>>(gcd, wsig, wgate, part, N, ncat1, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  gc_egrad_sum_kernel<<<(ncat1 * Ge + 255) / 256, 256, 0, st>>>(part, demb, nk, ncat1, Ge);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_lc_pack_launch(float* cat, float* wsig, float* wgate, int L, int Clc, int Cd, int pack, hipStream_t st) {
  lc_pack_kernel<<<grid_for((long)Clc * L * 2 * Cd), 256, 0, st>>>(cat, wsig, wgate, L, Clc, Cd, pack);
  LBWN_CHECK_LAUNCH();
  return 0;
}
