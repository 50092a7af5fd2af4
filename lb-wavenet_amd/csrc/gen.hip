// Cached single-step autoregressive generation (imodel.py:61-272).
//
// Per generated sample, all state stays on device so a chunk of steps can be captured in a
// hipGraph and replayed: the step counter, the per-layer lookback rings (the generation
// form of the D-separation cache: layer l keeps its last d inputs, slot t mod d, replacing
// imodel's shift-by-chunk buffers imodel.py:88-98, :190-207), the next input code, the
// teacher vector and a counter-based RNG.  One step =
//   gen_wave     one wave per stream, no barriers: PRE row (+bias), 50 × [dilated conv
//                (lane = output channel, 64-term dot over LDS broadcasts), gate (lane pairs),
//                residual], weights from a lane-coalesced image prefetched a layer ahead
//   gen_gemv × 3 K-split row-vector products with deterministic partial sums:
//                skip = z_cat·SKIPcat, h = relu(relu(skip + Σb)·POST1 + b1), logits = h·POST2
//   gen_sample   logits = Σ partials + b2; inverse-CDF draw with u = hash(seed, stream, step),
//                µ-law decode, next input = teacher[t] or the draw (imodel.py:167-187, :260-269)
#include <math.h>
#include <string.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {


// Wave-level LDS sync for single-wave workgroups: orders the wave's own LDS traffic without
// the vmcnt(0) that __syncthreads() implies (which would also wait for the next layer's
// weight prefetch, putting its L2 latency back on the chain).
LBWN_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Σ_q p[q·stride], q < n: independent loads in batches of 8 (a plain loop waits on each)
LBWN_DEV float sum_parts(const float* p, long stride, int n) {
  float s = 0.f;
  int q = 0;
  for (; q + 8 <= n; q += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = p[(q + i) * stride];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  for (; q < n; ++q) s += p[q * stride];
  return s;
}

LBWN_DEV long ring_offset(int l, int nbl, int B, int Cr) {
  const long s = (long)(l / nbl) * ((1L << nbl) - 1) + ((1L << (l % nbl)) - 1);
  return s * B * Cr;
}

// ---- per-stream wave chain ---------------------------------------------------------------
// One wave per stream, no barriers: lane o computes conv output o (sig 0-31 | gate 32-63) as
// a 64-term dot product over [x[t-d] | x[t]] (LDS broadcasts), the gate pairs lane o with
// lane o+32 (shuffle), the residual reads z back through wave-private LDS.  Weights come
// from a lane-coalesced per-layer image (packed once per gen_start) as 26 16-B loads per
// lane, prefetched one layer ahead into a register double buffer.
constexpr int GI_W = 16 * 64 * 4;           // conv: [kq 16][lane 64][4]  W[4kq+j][lane]
constexpr int GI_R = 8 * 64 * 4;            // residual: [cq 8][lane 64][4] RES[4cq+j][lane] (lane < 32)
constexpr int GIMG = GI_W + GI_R + 128;     // + conv bias [64] + residual bias [64]

struct LayerRegs {
  floatx4 w[16];
  floatx4 r[8];
  float bc, br, gc;
};

struct WaveK {
  const float* pre; const float* pre_b; const float* img; const float* gc_proj;
  float* rings; float* zcat; const long long* step; const int* code;
  int B, L, nbl, Cr, Cd, pre_bias;
};

LBWN_DEV void load_layer(LayerRegs& R, const WaveK& a, int l, int b, int lane) {
  const float* base = a.img + (long)l * GIMG;
#pragma unroll
  for (int kq = 0; kq < 16; ++kq) R.w[kq] = *(const floatx4*)(base + (kq * 64 + lane) * 4);
#pragma unroll
  for (int cq = 0; cq < 8; ++cq) R.r[cq] = *(const floatx4*)(base + GI_W + (cq * 64 + lane) * 4);
  R.bc = base[GI_W + GI_R + lane];
  R.br = base[GI_W + GI_R + 64 + lane];
  R.gc = a.gc_proj ? a.gc_proj[((long)l * a.B + b) * 64 + lane] : 0.f;
}

LBWN_DEV float dot4(const floatx4& w, const floatx4& x, float acc) {
  acc = fmaf(w[0], x[0], acc);
  acc = fmaf(w[1], x[1], acc);
  acc = fmaf(w[2], x[2], acc);
  return fmaf(w[3], x[3], acc);
}

__global__ __launch_bounds__(64) void gen_wave_kernel(WaveK a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* XP = sm;                    // [L][32] dilated taps of this step
  float* X = XP + a.L * 32;          // [32] current layer input
  float* Z = X + 32;                 // [32] gate output
  const int lane = threadIdx.x, b = blockIdx.x;
  const long t = *a.step;
  const int Cr = a.Cr, L = a.L;
  LayerRegs RA, RB;
  load_layer(RA, a, 0, b, lane);
  // every layer's tap: input of layer l at t - d_l (ring slot t mod d, zero-initialised).
  // d is a power of two: slot = t & (d-1); ring offsets accumulate (no integer division)
  {
    long roff = 0;
    int bl = 0;
    for (int l = 0; l < L; ++l) {
      const int d = 1 << bl;
      if ((lane >> 5) == (l & 1) && (lane & 31) < Cr) {
        const int c = lane & 31;
        XP[l * 32 + c] = a.rings[roff + ((long)b * d + (t & (d - 1))) * Cr + c];
      } else if ((lane >> 5) == (l & 1)) {
        XP[l * 32 + (lane & 31)] = 0.f;
      }
      roff += (long)d * a.B * Cr;
      bl = (bl + 1 == a.nbl) ? 0 : bl + 1;
    }
  }
  // step input: PRE row of the previous draw (+ PRE_BIAS); the zero vector at step 0
  float xr = 0.f;   // lane c < 32: x[c] of the current layer input
  if (lane < 32) {
    if (lane < Cr) {
      const int code = a.code[b];
      if (code >= 0) xr = a.pre[(long)code * Cr + lane];
      if (a.pre_bias && a.pre_b) xr += a.pre_b[lane];
    }
    X[lane] = xr;
  }
  wave_sync();

  long roff = 0;   // ring offset of layer l
  int bl = 0;      // l % nbl
  auto layer = [&](int l, LayerRegs& R, LayerRegs& N) {
    if (l + 1 < L) load_layer(N, a, l + 1, b, lane);
    const int d = 1 << bl;
    if (lane < Cr) a.rings[roff + ((long)b * d + (t & (d - 1))) * Cr + lane] = xr;
    roff += (long)d * a.B * Cr;
    bl = (bl + 1 == a.nbl) ? 0 : bl + 1;
    const float* xp = XP + l * 32;
    float acc0 = R.bc + R.gc, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
#pragma unroll
    for (int kq = 0; kq < 8; kq += 2) {
      acc0 = dot4(R.w[kq], *(const floatx4*)(xp + 4 * kq), acc0);
      acc1 = dot4(R.w[kq + 1], *(const floatx4*)(xp + 4 * kq + 4), acc1);
    }
#pragma unroll
    for (int kq = 0; kq < 8; kq += 2) {
      acc2 = dot4(R.w[8 + kq], *(const floatx4*)(X + 4 * kq), acc2);
      acc3 = dot4(R.w[8 + kq + 1], *(const floatx4*)(X + 4 * kq + 4), acc3);
    }
    const float v = (acc0 + acc1) + (acc2 + acc3);
    const float vg = __shfl_xor(v, 32);
    const float z = tanhf_(v) * sigmoidf_(vg);      // valid on lanes < 32 (padded channels: v = 0 -> z = 0)
    if (lane < a.Cd) a.zcat[(long)b * L * a.Cd + (long)l * a.Cd + lane] = z;
    if (lane < 32) Z[lane] = z;
    wave_sync();
    float r0 = R.br, r1 = 0.f;
#pragma unroll
    for (int cq = 0; cq < 8; cq += 2) {
      r0 = dot4(R.r[cq], *(const floatx4*)(Z + 4 * cq), r0);
      r1 = dot4(R.r[cq + 1], *(const floatx4*)(Z + 4 * cq + 4), r1);
    }
    xr += r0 + r1;
    if (lane < 32) X[lane] = xr;
    wave_sync();
  };
  for (int l = 0; l < L; l += 2) {
    layer(l, RA, RB);
    if (l + 1 < L) layer(l + 1, RB, RA);
  }
}

// per-layer lane-coalesced weight image (reference layouts in, GIMG floats per layer out)
__global__ void gen_pack_kernel(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                const float* res, const float* res_b, float* img, int Cr, int Cd) {
  const int l = blockIdx.x;
  float* o = img + (long)l * GIMG;
  for (int e = threadIdx.x; e < GIMG; e += blockDim.x) {
    float v = 0.f;
    if (e < GI_W) {
      const int kq = e / 256, lane = (e % 256) / 4, j = e % 4, k = 4 * kq + j;
      const int tap = k >> 5, in = k & 31, oc = lane & 31;
      if (in < Cr && oc < Cd) v = (lane < 32 ? sig : gate)[(long)l * 2 * Cr * Cd + (tap * Cr + in) * Cd + oc];
    } else if (e < GI_W + GI_R) {
      const int f = e - GI_W, cq = f / 256, lane = (f % 256) / 4, j = f % 4, c = 4 * cq + j;
      if (lane < Cr && c < Cd) v = res[(long)l * Cd * Cr + c * Cr + lane];
    } else {
      const int f = e - GI_W - GI_R;
      if (f < 64) {
        const float* bb = f < 32 ? sig_b : gate_b;
        if (bb && (f & 31) < Cd) v = bb[(long)l * Cd + (f & 31)];
      } else if (res_b && f - 64 < Cr) {
        v = res_b[(long)l * Cr + f - 64];
      }
    }
    o[e] = v;
  }
}

// ---- K-split row-vector GEMV --------------------------------------------------------------
// part[ks][b][n] = Σ_{k in slice ks} act(in[b][k])·W[k][n]: block = 64 columns (lane = n) ×
// one K slice, 4 waves over the slice's rows.  The input is either a plain [B][K] row buffer
// or the previous GEMV's partials, summed here in a fixed order (+ bias, relu): the chain of
// skip -> post1 -> post2 -> sample stays deterministic without atomics.
constexpr int GV_KSL_MAX = 64;   // K rows per slice (runtime KSL <= this, multiple of 4)

struct GemvK {
  const float* in; long ldin;                   // plain input rows, or
  const float* in_part; int in_parts;           // partials [in_parts][B][K]
  const float* in_bias; int relu_in;            // applied after the sum
  const float* W; long ldw;
  float* out_part;                              // [ceil(K/KSL)][B][N]
  int B, K, N, KSL;
};

__global__ __launch_bounds__(256) void gen_gemv_kernel(GemvK a) {
  __shared__ __attribute__((aligned(16))) float xs[16][GV_KSL_MAX];
  __shared__ float red[4][16][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int KSL = a.KSL, ks = blockIdx.y, k0 = ks * KSL, k1 = min(a.K, k0 + KSL);
  float wr[GV_KSL_MAX / 4];
#pragma unroll
  for (int i = 0; i < GV_KSL_MAX / 4; ++i) {
    const int k = k0 + w + 4 * i;
    wr[i] = (4 * i < KSL && k < k1 && n < a.N) ? a.W[(long)k * a.ldw + n] : 0.f;
  }
  for (int b0 = 0; b0 < a.B; b0 += 16) {
    const int nbb = min(16, a.B - b0);
    for (int e = tid; e < 16 * KSL; e += 256) {
      const int j = e / KSL, kk = e % KSL, k = k0 + kk;
      float v = 0.f;
      if (j < nbb && k < a.K) {
        if (a.in_part) {
          v = sum_parts(a.in_part + (long)(b0 + j) * a.K + k, (long)a.B * a.K, a.in_parts);
          if (a.in_bias) v += a.in_bias[k];
        } else {
          v = a.in[(long)(b0 + j) * a.ldin + k];
        }
        if (a.relu_in) v = fmaxf(v, 0.f);
      }
      xs[j][kk] = v;
    }
    __syncthreads();
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
    for (int i = 0; i < GV_KSL_MAX / 4; ++i)
      if (4 * i < KSL) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(xs[j][w + 4 * i], wr[i], acc[j]);
      }
#pragma unroll
    for (int j = 0; j < 16; ++j) red[w][j][lane] = acc[j];
    __syncthreads();
    for (int e = tid; e < 16 * 64; e += 256) {
      const int j = e >> 6, c = e & 63, nn = blockIdx.x * 64 + c;
      if (j < nbb && nn < a.N)
        a.out_part[((long)ks * a.B + b0 + j) * a.N + nn] = ((red[0][j][c] + red[1][j][c]) + red[2][j][c]) + red[3][j][c];
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
  float* logits; int Q, B;
  const float* log_part; int parts; const float* bias;   // logits = Σ parts + bias (written to logits)
  long long* step; int* code; const int* teacher; long long n_teacher;
  int* samples; float* wav; long long max_steps; unsigned long long seed;
};

// one block; wave w handles streams w, w+16, ...: softmax CDF in a fixed order, first k with
// cumsum(e)[k] > u·Σe (oracle/wavenet_ref.py sample_from_logits restates the same transform).
__global__ __launch_bounds__(1024) void gen_sample_kernel(SampleK a) {
  extern __shared__ float lgs[];   // [16][Q]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long t = *a.step;
  for (int b = w; b < a.B; b += 16) {
    float* lg = lgs + w * a.Q;
    for (int c = lane; c < a.Q; c += 64) {
      float v = sum_parts(a.log_part + (long)b * a.Q + c, (long)a.B * a.Q, a.parts);
      if (a.bias) v += a.bias[c];
      lg[c] = v;
      a.logits[(long)b * a.Q + c] = v;
    }
    wave_sync();
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
  size_t oRING, oZCAT, oSKP, oHP, oLGP, oLOG, oSTEP, oCODE, oTEACH, oSAMP, oWAV, oGCP, oBSUM, oGIMG, total;
  int ksl_skip, ks_skip, ks_h, ks_lg;
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
  LBWN_REQUIRE(a->n_blocks * a->n_block_layers * 32 * 4 + 256 <= 64 * 1024, "gen: too many layers for the tap cache");
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
  // K-split GEMV partials: skip (K = L·Cd, 64-row slices), post1 and post2 (32-row slices)
  p->ksl_skip = 64;
  p->ks_skip = (p->L * p->Cd + p->ksl_skip - 1) / p->ksl_skip;
  p->ks_h = (p->Cs + 31) / 32;
  p->ks_lg = (p->Cp + 31) / 32;
  p->oSKP = gcarve(cur, 4 * (size_t)p->ks_skip * B * p->Cs);
  p->oHP = gcarve(cur, 4 * (size_t)p->ks_h * B * p->Cp);
  p->oLGP = gcarve(cur, 4 * (size_t)p->ks_lg * B * p->Q);
  p->oLOG = gcarve(cur, 4 * (size_t)B * p->Q);
  p->oSTEP = gcarve(cur, 8);
  p->oCODE = gcarve(cur, 4 * (size_t)B);
  p->oTEACH = gcarve(cur, 4 * (size_t)std::max<int64_t>(1, max_teacher));
  p->oSAMP = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oWAV = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oGCP = gcarve(cur, 4 * (size_t)p->L * B * 64);
  p->oBSUM = gcarve(cur, 4 * (size_t)p->Cs);
  p->oGIMG = gcarve(cur, 4 * (size_t)p->L * GIMG);
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
  gen_pack_kernel<<<p->L, 256, 0, st>>>(P->sig, P->gate, P->sig_b, P->gate_b, P->res, P->res_b, gat<float>(ws, p->oGIMG),
                                        p->Cr, p->Cd);
  LBWN_CHECK_LAUNCH();
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
  WaveK c;
  c.pre = P->pre; c.pre_b = P->pre_b; c.img = gat<float>(ws, p->oGIMG);
  c.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
  c.rings = gat<float>(ws, p->oRING); c.zcat = gat<float>(ws, p->oZCAT);
  c.step = gat<long long>(ws, p->oSTEP); c.code = gat<int>(ws, p->oCODE);
  c.B = p->B; c.L = p->L; c.nbl = p->nbl; c.Cr = p->Cr; c.Cd = p->Cd; c.pre_bias = p->pre_bias;
  const size_t wave_lds = 4 * ((size_t)p->L * 32 + 64);
  // skip = z_cat·SKIPcat (+Σb and relu applied by the consumer), h = relu(relu(skip)·POST1 + b1),
  // logits = h·POST2 + b2 (summed in the sampler)
  GemvK sk, p1, p2;
  memset(&sk, 0, sizeof(sk));
  sk.in = c.zcat; sk.ldin = (long)p->L * p->Cd; sk.W = P->skip; sk.ldw = p->Cs; sk.out_part = gat<float>(ws, p->oSKP);
  sk.B = p->B; sk.K = p->L * p->Cd; sk.N = p->Cs; sk.KSL = p->ksl_skip;
  p1 = sk;
  p1.in = nullptr; p1.in_part = sk.out_part; p1.in_parts = p->ks_skip; p1.in_bias = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr;
  p1.relu_in = 1; p1.W = P->post1; p1.ldw = p->Cp; p1.out_part = gat<float>(ws, p->oHP); p1.K = p->Cs; p1.N = p->Cp; p1.KSL = 32;
  p2 = p1;
  p2.in_part = p1.out_part; p2.in_parts = p->ks_h; p2.in_bias = P->post1_b; p2.relu_in = 1;
  p2.W = P->post2; p2.ldw = p->Q; p2.out_part = gat<float>(ws, p->oLGP); p2.K = p->Cp; p2.N = p->Q; p2.KSL = 32;
  SampleK sm;
  sm.logits = gat<float>(ws, p->oLOG); sm.Q = p->Q; sm.B = p->B;
  sm.log_part = p2.out_part; sm.parts = p->ks_lg; sm.bias = P->post2_b;
  sm.step = gat<long long>(ws, p->oSTEP); sm.code = gat<int>(ws, p->oCODE);
  sm.teacher = gat<int>(ws, p->oTEACH); sm.n_teacher = p->n_teacher; sm.samples = gat<int>(ws, p->oSAMP);
  sm.wav = gat<float>(ws, p->oWAV); sm.max_steps = p->max_steps; sm.seed = p->seed;
  const dim3 gsk((sk.N + 63) / 64, p->ks_skip), gp1((p1.N + 63) / 64, (p1.K + 31) / 32), gp2((p2.N + 63) / 64, (p2.K + 31) / 32);
  const size_t sample_lds = 4 * (size_t)16 * p->Q;
  for (int i = 0; i < n_steps; ++i) {
    gen_wave_kernel<<<p->B, 64, wave_lds, st>>>(c);
    gen_gemv_kernel<<<gsk, 256, 0, st>>>(sk);
    gen_gemv_kernel<<<gp1, 256, 0, st>>>(p1);
    gen_gemv_kernel<<<gp2, 256, 0, st>>>(p2);
    gen_sample_kernel<<<1, 1024, sample_lds, st>>>(sm);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}
