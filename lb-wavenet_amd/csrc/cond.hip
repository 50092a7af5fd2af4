// Global / local conditioning (tmodel.py:68-83, :92-114, :150-160).
//
// GC: the per-layer term GC_EMBED[ids]·GC_k_l depends on the position only through its
// voice id, so it is a lookup in a per-step table GCTAB[l][c][sig Cd | gate Cd] =
// GC_EMBED[c]·[GC_SIGNAL_l | GC_GATE_l]; the layer kernels add row ids[m].  Backward: the
// layer kernels scatter-add dv rows into GCD[l][c][2Cd] (per voice id), and
//   dGC_SIGNAL_l = GC_EMBEDᵀ·GCD_l[:, :Cd],  dGC_EMBED = Σ_l GCD_l·[GC_SIGNAL_l | GC_GATE_l]ᵀ.
// LC: the per-layer projections LC_SIGNAL_l / LC_GATE_l are packed side by side into one
// [Clc][L·2Cd] matrix so the whole conditioning input is ONE GEMM lc·LCcat (engine.cpp).
#include "common.h"
#include "kernels.h"

namespace {

// out[l][c][s·Cd + o] = Σ_e emb[c][e] · W_s[l][e][o]
__global__ void gc_table_kernel(const float* __restrict__ emb, const float* __restrict__ wsig,
                                const float* __restrict__ wgate, float* __restrict__ out, int L, int ncat1, int Ge,
                                int Cd) {
  const long total = (long)L * ncat1 * 2 * Cd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i % (2 * Cd)), c = (int)((i / (2 * Cd)) % ncat1), l = (int)(i / (2L * Cd * ncat1));
    const float* W = (n < Cd ? wsig : wgate) + (long)l * Ge * Cd + (n % Cd);
    const float* e = emb + (long)c * Ge;
    float acc = 0.f;
    for (int k = 0; k < Ge; ++k) acc += e[k] * W[(long)k * Cd];
    out[i] = acc;
  }
}

// dW_s[l][e][o] = Σ_c emb[c][e] · GCD[l][c][s·Cd + o]
__global__ void gc_wgrad_kernel(const float* __restrict__ emb, const float* __restrict__ gcd, float* __restrict__ dsig,
                                float* __restrict__ dgate, int L, int ncat1, int Ge, int Cd) {
  const long total = (long)L * 2 * Ge * Cd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int o = (int)(i % Cd), e = (int)((i / Cd) % Ge), s = (int)((i / ((long)Cd * Ge)) % 2),
              l = (int)(i / (2L * Ge * Cd));
    const float* g = gcd + (long)l * ncat1 * 2 * Cd + s * Cd + o;
    float acc = 0.f;
    for (int c = 0; c < ncat1; ++c) acc += emb[(long)c * Ge + e] * g[(long)c * 2 * Cd];
    (s == 0 ? dsig : dgate)[(long)l * Ge * Cd + (long)e * Cd + o] = acc;
  }
}

// dEMB[c][e] = Σ_l Σ_n GCD[l][c][n] · W_{n<Cd ? sig : gate}[l][e][n % Cd]; one block per c,
// one thread per (e, partial over n), reduced in LDS.
__global__ __launch_bounds__(256) void gc_egrad_kernel(const float* __restrict__ gcd, const float* __restrict__ wsig,
                                                       const float* __restrict__ wgate, float* __restrict__ demb,
                                                       int L, int ncat1, int Ge, int Cd) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  for (int e0 = 0; e0 < Ge; ++e0) {
    float acc = 0.f;
    for (long j = threadIdx.x; j < (long)L * 2 * Cd; j += 256) {
      const int l = (int)(j / (2 * Cd)), n = (int)(j % (2 * Cd));
      const float* W = (n < Cd ? wsig : wgate) + (long)l * Ge * Cd + (long)e0 * Cd + (n % Cd);
      acc += gcd[((long)l * ncat1 + c) * 2 * Cd + n] * *W;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) demb[(long)c * Ge + e0] = red[0];
    __syncthreads();
  }
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

int lbwn_gc_table_launch(const float* emb, const float* wsig, const float* wgate, float* out, int L, int ncat1,
                         int Ge, int Cd, hipStream_t st) {
  gc_table_kernel<<<grid_for((long)L * ncat1 * 2 * Cd), 256, 0, st>>>(emb, wsig, wgate, out, L, ncat1, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_gc_grad_launch(const float* emb, const float* wsig, const float* wgate, const float* gcd, float* demb,
                        float* dsig, float* dgate, int L, int ncat1, int Ge, int Cd, hipStream_t st) {
  gc_wgrad_kernel<<<grid_for((long)L * 2 * Ge * Cd), 256, 0, st>>>(emb, gcd, dsig, dgate, L, ncat1, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  gc_egrad_kernel<<<ncat1, 256, 0, st>>>(gcd, wsig, wgate, demb, L, ncat1, Ge, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_lc_pack_launch(float* cat, float* wsig, float* wgate, int L, int Clc, int Cd, int pack, hipStream_t st) {
  lc_pack_kernel<<<grid_for((long)Clc * L * 2 * Cd), 256, 0, st>>>(cat, wsig, wgate, L, Clc, Cd, pack);
  LBWN_CHECK_LAUNCH();
  return 0;
}
