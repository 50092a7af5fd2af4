// Cached single-step autoregressive generation (imodel.py:61-272).
//
// Per generated sample, all state stays on device so a chunk of steps can be captured in a
// hipGraph and replayed: the step counter, the per-layer lookback rings (the generation
// form of the D-separation cache: layer l keeps its last d inputs, slot t mod d, replacing
// imodel's shift-by-chunk buffers imodel.py:88-98, :190-207), the next input code, the
// teacher vector and a counter-based RNG.  One step =
//   gen_chain   1 workgroup per 16 streams: PRE row (+bias), 50 × [dilated conv (VALU; B is
//               ~10 so a 32-wide MFMA tile would be mostly padding), gate, residual], z_cat out
//   gen_rowvec  × 3: skip = z_cat·SKIPcat + Σb, h = relu(relu(skip)·POST1 + b1),
//               logits = h·POST2 + b2 (weights L2-resident across steps)
//   gen_sample  inverse-CDF draw of softmax(logits) with u = hash(seed, stream, step),
//               µ-law decode, next input = teacher[t] or the draw (imodel.py:167-187, :260-269)
#include <math.h>
#include <string.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int GB = 16;                 // streams per chain workgroup
constexpr int RV_MAXI = 32;            // row-vector GEMM: K <= 64·32 = 2048
constexpr int WIMG_G = 64 * 64 + 32 * 32 + 96;  // conv W[k][o] (64×64) | RES[c][o] (32×32) | b_conv[64] | b_res[32]

struct ChainK {
  const float* pre; const float* pre_b;
  const float* sig; const float* gate; const float* sig_b; const float* gate_b;
  const float* res; const float* res_b;
  const float* gc_proj;   // [L][B][64] or null
  float* rings;           // packed per layer [B][d][Cr]
  float* zcat;            // [B][L*Cd]
  const long long* step;  // current step t
  int* code;              // [B] input code for this step (-1 = zero vector)
  int B, L, nbl, Cr, Cd, Q, pre_bias;
};

LBWN_DEV long ring_offset(int l, int nbl, int B, int Cr) {
  const long s = (long)(l / nbl) * ((1L << nbl) - 1) + ((1L << (l % nbl)) - 1);
  return s * B * Cr;
}

// stage layer l's weights (reference layouts) into registers -> LDS image
struct WStage {
  static constexpr int N = (WIMG_G + 1023) / 1024;  // 6 per thread
  float v[N];
  LBWN_DEV void load(const ChainK& a, int l, int tid) {
    const int Cr = a.Cr, Cd = a.Cd;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int e = tid + 1024 * i;
      float x = 0.f;
      if (e < 64 * 64) {
        const int k = e >> 6, o = e & 63, tap = k >> 5, in = k & 31, oc = o & 31;
        if (in < Cr && oc < Cd) x = (o < 32 ? a.sig : a.gate)[(long)l * 2 * Cr * Cd + (tap * Cr + in) * Cd + oc];
      } else if (e < 64 * 64 + 32 * 32) {
        const int f = e - 64 * 64, c = f >> 5, o = f & 31;
        if (c < Cd && o < Cr) x = a.res[(long)l * Cd * Cr + c * Cr + o];
      } else if (e < WIMG_G) {
        const int f = e - 64 * 64 - 32 * 32;
        if (f < 64) {
          const float* bb = f < 32 ? a.sig_b : a.gate_b;
          if (bb && (f & 31) < Cd) x = bb[(long)l * Cd + (f & 31)];
        } else if (a.res_b && f - 64 < Cr) {
          x = a.res_b[(long)l * Cr + f - 64];
        }
      }
      v[i] = x;
    }
  }
  LBWN_DEV void store(float* W, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int e = tid + 1024 * i;
      if (e < WIMG_G) W[e] = v[i];
    }
  }
};

// LDS: all L layers' lookback taps (read once, up front), 2 weight images, x/z rows,
// conv partials over 2 K-halves.  GBS streams per workgroup (16, or 8 for deep stacks).
template <int GBS>
__global__ __launch_bounds__(1024) void gen_chain_kernel(ChainK a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Wb0 = sm;
  float* Wb1 = sm + WIMG_G;
  float* X = Wb1 + WIMG_G;          // [GBS][32]
  float* Z = X + GBS * 32;          // [GBS][32]
  float* P = Z + GBS * 32;          // [2][GBS][64]
  float* PV = P + 2 * GBS * 64;     // [L][GBS][32]
  const int tid = threadIdx.x;
  const int b0 = blockIdx.x * GBS;
  const int nb = min(GBS, a.B - b0);
  const long t = *a.step;
  const int Cr = a.Cr, Cd = a.Cd, L = a.L;

  WStage ws;
  ws.load(a, 0, tid);
  // every layer's prev tap: input of layer l at t - d_l (ring slot t mod d_l, zero-initialised)
  {
    const int n = L * GBS * 32;
    for (int base = tid; base < n; base += 1024 * 8) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = base + 1024 * i;
        v[i] = 0.f;
        if (e < n) {
          const int l = e / (GBS * 32), r = e % (GBS * 32), b = r >> 5, c = r & 31;
          const int d = 1 << (l % a.nbl);
          if (b < nb && c < Cr) v[i] = a.rings[ring_offset(l, a.nbl, a.B, Cr) + ((long)(b0 + b) * d + (t % d)) * Cr + c];
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (base + 1024 * i < n) PV[base + 1024 * i] = v[i];
    }
  }
  // input z0 = onehot(code)·PRE (+ PRE_BIAS): zero vector at step 0 (imodel.py:61-79)
  if (tid < GBS * 32) {
    const int b = tid >> 5, c = tid & 31;
    float v = 0.f;
    if (b < nb && c < Cr) {
      const int code = a.code[b0 + b];
      if (code >= 0) v = a.pre[(long)code * Cr + c];
      if (a.pre_bias && a.pre_b) v += a.pre_b[c];
    }
    X[tid] = v;
  }
  ws.store(Wb0, tid);
  __syncthreads();

  constexpr int SPG = GBS / 8;   // streams per conv thread
  for (int l = 0; l < L; ++l) {
    const float* W = (l & 1) ? Wb1 : Wb0;
    float* Wn = (l & 1) ? Wb0 : Wb1;
    const float* pv = PV + l * GBS * 32;
    if (l + 1 < L) ws.load(a, l + 1, tid);   // next layer's weights land during this layer
    // ring write: this layer's input becomes the tap of step t + d (slot t mod d)
    if (tid < GBS * 32) {
      const int b = tid >> 5, c = tid & 31;
      const int d = 1 << (l % a.nbl);
      if (b < nb && c < Cr)
        a.rings[ring_offset(l, a.nbl, a.B, Cr) + ((long)(b0 + b) * d + (t % d)) * Cr + c] = X[tid];
    }
    // conv partials: thread (o, K-half kh, stream group bg): SPG streams × 32 k
    {
      const int o = tid & 63, kh = (tid >> 6) & 1, bg = tid >> 7;
      const float* xin = kh ? X : pv;
      float acc[SPG];
#pragma unroll
      for (int j = 0; j < SPG; ++j) acc[j] = 0.f;
#pragma unroll 8
      for (int k = 0; k < 32; ++k) {
        const float w = W[(kh * 32 + k) * 64 + o];
#pragma unroll
        for (int j = 0; j < SPG; ++j) acc[j] = fmaf(xin[(bg * SPG + j) * 32 + k], w, acc[j]);
      }
#pragma unroll
      for (int j = 0; j < SPG; ++j) P[(kh * GBS + bg * SPG + j) * 64 + o] = acc[j];
    }
    __syncthreads();
    // gate
    if (tid < GBS * 32) {
      const int b = tid >> 5, c = tid & 31;
      const float* bs = W + 64 * 64 + 32 * 32;
      float vs = bs[c] + P[b * 64 + c] + P[(GBS + b) * 64 + c];
      float vg = bs[32 + c] + P[b * 64 + 32 + c] + P[(GBS + b) * 64 + 32 + c];
      if (a.gc_proj && b < nb) {
        const float* g = a.gc_proj + ((long)l * a.B + b0 + b) * 64;
        vs += g[c];
        vg += g[32 + c];
      }
      const float z = (c < Cd && b < nb) ? tanhf_(vs) * sigmoidf_(vg) : 0.f;
      Z[tid] = z;
      if (b < nb && c < Cd) a.zcat[(long)(b0 + b) * L * Cd + l * Cd + c] = z;
    }
    __syncthreads();
    // residual: x += z·RES + b
    if (tid < GBS * 32) {
      const int b = tid >> 5, o = tid & 31;
      const float* R = W + 64 * 64;
      float r = W[64 * 64 + 32 * 32 + 64 + o];   // b_res
#pragma unroll 8
      for (int c = 0; c < 32; ++c) r = fmaf(Z[b * 32 + c], R[c * 32 + o], r);
      X[tid] += r;
    }
    if (l + 1 < L) ws.store(Wn, tid);
    __syncthreads();
  }
}

size_t chain_lds_bytes(int gbs, int L) { return 4 * (size_t)(2 * WIMG_G + 2 * gbs * 32 + 2 * gbs * 64 + (size_t)L * gbs * 32); }

// out[b][n] = epi( Σ_k act(in[b][k])·W[k][n] + bias ), b < B (≤ 64 per launch row loop),
// block = 4 columns; thread (c = tid & 3, ks = tid >> 2): K slice, all streams.
struct RowK {
  const float* in; long ldin; const float* W; long ldw; float* out; long ldout;
  const float* bias;                  // [N] nullable
  int B, K, N, relu_in, relu_out;
};

__global__ __launch_bounds__(256) void gen_rowvec_kernel(RowK a) {
  extern __shared__ __attribute__((aligned(16))) float xin[];   // [16][K] (act applied)
  __shared__ float red[64][4][17];
  const int c = threadIdx.x & 3, ks = threadIdx.x >> 2;  // 64 K slices
  const int n = blockIdx.x * 4 + c;
  float acc[16];
  // every weight of this thread's K slice is issued first (K <= 64·RV_MAXI); it lands while
  // the activations are staged
  float wr[RV_MAXI];
#pragma unroll
  for (int i = 0; i < RV_MAXI; ++i) {
    const int k = ks + 64 * i;
    wr[i] = (n < a.N && k < a.K) ? a.W[(long)k * a.ldw + n] : 0.f;
  }
  for (int bb0 = 0; bb0 < a.B; bb0 += 16) {
    const int nbb = min(16, a.B - bb0);
    {
      const int nf4 = 16 * a.K / 4;   // K % 4 == 0, ldin % 4 == 0
      for (int base = threadIdx.x; base < nf4; base += 256 * 8) {
        floatx4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = base + 256 * i;
          v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
          if (e < nf4) {
            const int j = (4 * e) / a.K, k = (4 * e) % a.K;
            if (j < nbb) {
              v[i] = *(const floatx4*)(a.in + (long)(bb0 + j) * a.ldin + k);
              if (a.relu_in) {
                v[i][0] = fmaxf(v[i][0], 0.f); v[i][1] = fmaxf(v[i][1], 0.f);
                v[i][2] = fmaxf(v[i][2], 0.f); v[i][3] = fmaxf(v[i][3], 0.f);
              }
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (base + 256 * i < nf4) *(floatx4*)(xin + 4 * (base + 256 * i)) = v[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    if (n < a.N) {
#pragma unroll
      for (int i = 0; i < RV_MAXI; ++i) {
        const int k = ks + 64 * i;
        if (k < a.K) {
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[j] = fmaf(xin[j * a.K + k], wr[i], acc[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) red[ks][c][j] = acc[j];
    __syncthreads();
    if (threadIdx.x < 64) {
      const int cc = threadIdx.x & 3, j = threadIdx.x >> 2;
      const int nn = blockIdx.x * 4 + cc;
      if (nn < a.N && j < nbb) {
        float s = a.bias ? a.bias[nn] : 0.f;
        for (int q = 0; q < 64; ++q) s += red[q][cc][j];
        if (a.relu_out) s = fmaxf(s, 0.f);
        a.out[(long)(bb0 + j) * a.ldout + nn] = s;
      }
    }
    __syncthreads();
  }
}

LBWN_DEV uint64_t splitmix(uint64_t seed, uint64_t stream, uint64_t step) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ULL + (stream << 32) + step + 0x632BE59BD9B4E019ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct SampleK {
  const float* logits; int Q, B;
  long long* step; int* code; const int* teacher; long long n_teacher;
  int* samples; float* wav; long long max_steps; unsigned long long seed;
};

// one block; wave w handles streams w, w+16, ...: softmax CDF in a fixed order, first k with
// cumsum(e)[k] > u·Σe (oracle/wavenet_ref.py sample_from_logits restates the same transform).
__global__ __launch_bounds__(1024) void gen_sample_kernel(SampleK a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long t = *a.step;
  for (int b = w; b < a.B; b += 16) {
    const float* lg = a.logits + (long)b * a.Q;
    float mx = -INFINITY;
    for (int c = lane; c < a.Q; c += 64) mx = fmaxf(mx, lg[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    // each lane owns a contiguous run of Q/64 codes: local sums, then an exclusive scan
    const int per = (a.Q + 63) / 64, c0 = lane * per;
    float loc = 0.f;
    for (int j = 0; j < per; ++j)
      if (c0 + j < a.Q) loc += expf(lg[c0 + j] - mx);
    float incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const float total = __shfl(incl, 63);
    const float excl = incl - loc;
    const uint64_t h = splitmix(a.seed, (uint64_t)b, (uint64_t)t);
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    const float target = u * total;
    // lane whose run contains the crossing point
    int found = a.Q;
    if (excl <= target && target < incl) {
      float run = excl;
      for (int j = 0; j < per; ++j) {
        if (c0 + j >= a.Q) break;
        run += expf(lg[c0 + j] - mx);
        if (run > target) { found = c0 + j; break; }
      }
      if (found == a.Q) found = min(c0 + per, a.Q) - 1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) found = min(found, __shfl_xor(found, o));
    if (found >= a.Q) found = a.Q - 1;
    if (lane == 0) {
      if (t < a.max_steps) {
        a.samples[(long)b * a.max_steps + t] = found;
        const float mu = (float)(a.Q - 1), inv = 1.f / mu;               // ops.py:12-20
        const float aa = (2.f * (float)found - 1.f) * inv - 1.f;
        const float sg = aa > 0.f ? 1.f : (aa < 0.f ? -1.f : 0.f);
        a.wav[(long)b * a.max_steps + t] = sg * (powf(1.f + mu, fabsf(aa)) - 1.f) * inv;
      }
      a.code[b] = (t < a.n_teacher) ? a.teacher[t] : found;              // imodel.py:260-269
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) *a.step = t + 1;
}

// gc_proj[l][b][o] = GC_EMBED[gc_id[b]] · [GC_SIGNAL_l | GC_GATE_l]  (imodel.py:53-56, :113-118)
__global__ void gen_gc_proj_kernel(const float* emb, const float* gsig, const float* ggate, const int* ids,
                                   float* out, int B, int Ge, int Cd) {
  const int l = blockIdx.x;
  for (int e = threadIdx.x; e < B * 64; e += blockDim.x) {
    const int b = e / 64, o = e % 64, oc = o & 31;
    float s = 0.f;
    if (oc < Cd) {
      const float* G = (o < 32 ? gsig : ggate) + (long)l * Ge * Cd;
      const float* em = emb + (long)ids[b] * Ge;
      for (int k = 0; k < Ge; ++k) s += em[k] * G[k * Cd + oc];
    }
    out[((long)l * B + b) * 64 + o] = s;
  }
}

__global__ void gen_reset_kernel(float* rings, long n_ring, int* code, int B, long long* step) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n_ring; e += (long)gridDim.x * blockDim.x)
    rings[e] = 0.f;
  if (blockIdx.x == 0) {
    for (int b = threadIdx.x; b < B; b += blockDim.x) code[b] = -1;
    if (threadIdx.x == 0) *step = 0;
  }
}

}  // namespace

// ---- host side: generation plan ----------------------------------------------------------

#include "../../include/lbwn.h"

struct lbwn_gen_plan {
  lbwn_arch a;
  int B, L, nbl, Cr, Cd, Cs, Cp, Q;
  long long max_steps;
  size_t oRING, oZCAT, oSKIP, oH, oLOG, oSTEP, oCODE, oTEACH, oSAMP, oWAV, oGCP, oBSUM, total;
  long n_ring;
  long long n_teacher, max_teacher;
  unsigned long long seed;
  int pre_bias;
};

static size_t gcarve(size_t& cur, size_t bytes) {
  size_t o = cur;
  cur += (bytes + 255) / 256 * 256;
  return o;
}

extern "C" int lbwn_gen_plan_create(const lbwn_arch* a, int B, int64_t max_steps, int64_t max_teacher,
                                    lbwn_gen_plan** out) {
  LBWN_REQUIRE(a && out && B >= 1 && max_steps >= 1 && max_teacher >= 0, "gen_plan_create: bad arguments");
  LBWN_REQUIRE(a->n_res <= 32 && a->n_dil <= 32, "gen: n_res/n_dil must be <= 32");
  LBWN_REQUIRE(a->n_skip % 4 == 0 && a->n_post % 4 == 0 && ((long)a->n_blocks * a->n_block_layers * a->n_dil) % 4 == 0,
               "gen: row-vector GEMM needs K %% 4 == 0");
  LBWN_REQUIRE((long)a->n_blocks * a->n_block_layers * a->n_dil <= 2048 && a->n_skip <= 2048 && a->n_post <= 2048,
               "gen: row-vector GEMM K too large for LDS staging");
  LBWN_REQUIRE(a->n_lc_out == 0, "gen: local conditioning is not supported by the cached generator "
                                 "(imodel.py has no LC path)");
  lbwn_gen_plan* p = new lbwn_gen_plan();
  p->a = *a;
  p->B = B;
  p->nbl = a->n_block_layers;
  p->L = a->n_blocks * a->n_block_layers;
  p->Cr = a->n_res; p->Cd = a->n_dil; p->Cs = a->n_skip; p->Cp = a->n_post; p->Q = a->n_quant;
  p->max_steps = max_steps;
  p->max_teacher = max_teacher;
  long dsum = (long)a->n_blocks * ((1L << a->n_block_layers) - 1);
  p->n_ring = dsum * B * p->Cr;
  size_t cur = 0;
  p->oRING = gcarve(cur, 4 * (size_t)p->n_ring);
  p->oZCAT = gcarve(cur, 4 * (size_t)B * p->L * p->Cd);
  p->oSKIP = gcarve(cur, 4 * (size_t)B * p->Cs);
  p->oH = gcarve(cur, 4 * (size_t)B * p->Cp);
  p->oLOG = gcarve(cur, 4 * (size_t)B * p->Q);
  p->oSTEP = gcarve(cur, 8);
  p->oCODE = gcarve(cur, 4 * (size_t)B);
  p->oTEACH = gcarve(cur, 4 * (size_t)std::max<int64_t>(1, max_teacher));
  p->oSAMP = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oWAV = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oGCP = gcarve(cur, 4 * (size_t)p->L * B * 64);
  p->oBSUM = gcarve(cur, 4 * (size_t)p->Cs);
  p->total = cur;
  *out = p;
  return 0;
}

extern "C" void lbwn_gen_plan_destroy(lbwn_gen_plan* p) { delete p; }
extern "C" size_t lbwn_gen_workspace_bytes(const lbwn_gen_plan* p) { return p ? p->total : 0; }

extern "C" int lbwn_gen_tensor(const lbwn_gen_plan* p, const char* name, size_t* off, size_t* bytes) {
  LBWN_REQUIRE(p && name && off && bytes, "gen_tensor: null argument");
  const size_t B = p->B;
  if (!strcmp(name, "samples")) { *off = p->oSAMP; *bytes = 4 * B * p->max_steps; }
  else if (!strcmp(name, "wav")) { *off = p->oWAV; *bytes = 4 * B * p->max_steps; }
  else if (!strcmp(name, "logits")) { *off = p->oLOG; *bytes = 4 * B * p->Q; }
  else if (!strcmp(name, "step")) { *off = p->oSTEP; *bytes = 8; }
  else if (!strcmp(name, "rings")) { *off = p->oRING; *bytes = 4 * (size_t)p->n_ring; }
  else if (!strcmp(name, "teacher")) { *off = p->oTEACH; *bytes = 4 * (size_t)std::max<long long>(1, p->n_teacher); }
  else LBWN_REQUIRE(false, "gen_tensor: unknown tensor '%s'", name);
  return 0;
}

template <typename T>
static T* gat(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

extern "C" int lbwn_gen_start(lbwn_gen_plan* p, const lbwn_params* P, void* ws, const int* gc_ids,
                              const int* teacher, int64_t n_teacher, uint64_t seed, int pre_bias, void* stream) {
  LBWN_REQUIRE(p && P && ws, "gen_start: null argument");
  LBWN_REQUIRE(p->a.n_gc_embed == 0 || gc_ids, "gen_start: GC arch needs gc_ids [B]");
  LBWN_REQUIRE(!teacher || (n_teacher >= 0 && n_teacher <= p->max_teacher),
               "gen_start: teacher length %lld exceeds plan capacity %lld", (long long)n_teacher, p->max_teacher);
  hipStream_t st = (hipStream_t)stream;
  p->n_teacher = teacher ? n_teacher : 0;
  p->seed = seed;
  p->pre_bias = pre_bias;
  gen_reset_kernel<<<256, 256, 0, st>>>(gat<float>(ws, p->oRING), p->n_ring, gat<int>(ws, p->oCODE), p->B,
                                        gat<long long>(ws, p->oSTEP));
  LBWN_CHECK_LAUNCH();
  if (p->n_teacher > 0) {
    hipError_t e = hipMemcpyAsync(gat<int>(ws, p->oTEACH), teacher, 4 * (size_t)p->n_teacher, hipMemcpyDeviceToDevice,
                                  st);
    LBWN_REQUIRE(e == hipSuccess, "gen_start: teacher copy failed: %s", hipGetErrorString(e));
  }
  if (P->skip_b) {
    if (int e = lbwn_sum_bias_launch(P->skip_b, p->L, p->Cs, gat<float>(ws, p->oBSUM), st)) return e;
  }
  if (p->a.n_gc_embed > 0) {
    gen_gc_proj_kernel<<<p->L, 256, 0, st>>>(P->gc_embed, P->gc_sig, P->gc_gate, gc_ids, gat<float>(ws, p->oGCP),
                                             p->B, p->a.n_gc_embed, p->Cd);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lbwn_gen_run(lbwn_gen_plan* p, const lbwn_params* P, void* ws, int n_steps, void* stream) {
  LBWN_REQUIRE(p && P && ws && n_steps >= 0, "gen_run: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  ChainK c;
  c.pre = P->pre; c.pre_b = P->pre_b; c.sig = P->sig; c.gate = P->gate; c.sig_b = P->sig_b; c.gate_b = P->gate_b;
  c.res = P->res; c.res_b = P->res_b;
  c.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
  c.rings = gat<float>(ws, p->oRING); c.zcat = gat<float>(ws, p->oZCAT);
  c.step = gat<long long>(ws, p->oSTEP); c.code = gat<int>(ws, p->oCODE);
  c.B = p->B; c.L = p->L; c.nbl = p->nbl; c.Cr = p->Cr; c.Cd = p->Cd; c.Q = p->Q; c.pre_bias = p->pre_bias;
  RowK sk, p1, p2;
  sk.in = c.zcat; sk.ldin = (long)p->L * p->Cd; sk.W = P->skip; sk.ldw = p->Cs; sk.out = gat<float>(ws, p->oSKIP);
  sk.ldout = p->Cs; sk.bias = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr; sk.B = p->B; sk.K = p->L * p->Cd; sk.N = p->Cs;
  sk.relu_in = 0; sk.relu_out = 0;
  p1.in = sk.out; p1.ldin = p->Cs; p1.W = P->post1; p1.ldw = p->Cp; p1.out = gat<float>(ws, p->oH); p1.ldout = p->Cp;
  p1.bias = P->post1_b; p1.B = p->B; p1.K = p->Cs; p1.N = p->Cp; p1.relu_in = 1; p1.relu_out = 1;
  p2.in = p1.out; p2.ldin = p->Cp; p2.W = P->post2; p2.ldw = p->Q; p2.out = gat<float>(ws, p->oLOG); p2.ldout = p->Q;
  p2.bias = P->post2_b; p2.B = p->B; p2.K = p->Cp; p2.N = p->Q; p2.relu_in = 0; p2.relu_out = 0;
  SampleK sm;
  sm.logits = p2.out; sm.Q = p->Q; sm.B = p->B; sm.step = gat<long long>(ws, p->oSTEP); sm.code = c.code;
  sm.teacher = gat<int>(ws, p->oTEACH); sm.n_teacher = p->n_teacher; sm.samples = gat<int>(ws, p->oSAMP);
  sm.wav = gat<float>(ws, p->oWAV); sm.max_steps = p->max_steps; sm.seed = p->seed;
  const bool wide = chain_lds_bytes(16, p->L) <= 160 * 1024;
  const int gbs = wide ? 16 : 8;
  LBWN_REQUIRE(chain_lds_bytes(gbs, p->L) <= 160 * 1024, "gen: too many layers for the LDS tap cache");
  const int gchain = (p->B + gbs - 1) / gbs;
  const size_t lds = chain_lds_bytes(gbs, p->L);
  for (int i = 0; i < n_steps; ++i) {
    if (wide) gen_chain_kernel<16><<<gchain, 1024, lds, st>>>(c);
    else gen_chain_kernel<8><<<gchain, 1024, lds, st>>>(c);
    gen_rowvec_kernel<<<(sk.N + 3) / 4, 256, 64 * sk.K, st>>>(sk);
    gen_rowvec_kernel<<<(p1.N + 3) / 4, 256, 64 * p1.K, st>>>(p1);
    gen_rowvec_kernel<<<(p2.N + 3) / 4, 256, 64 * p2.K, st>>>(p2);
    gen_sample_kernel<<<1, 1024, 0, st>>>(sm);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}
