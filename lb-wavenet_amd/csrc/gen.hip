// Cached single-step autoregressive generation (imodel.py:61-272).
//
// All state stays on device, so a chunk of steps can be captured in a hipGraph and replayed:
// the step counter, the per-layer lookback rings (the generation form of the D-separation
// cache: layer l keeps its last d inputs, slot t mod d, replacing imodel's shift-by-chunk
// buffers imodel.py:88-98, :190-207), the next input code, the teacher vector and a
// counter-based RNG.  Two execution forms, chosen at plan creation:
//   persistent (the default while its blocks fit: groups of <= 16 streams, each group with its
//     own head blocks, B <= 80 on 256 CUs): ONE launch per run, gen_persist_kernel — chain
//     blocks (one per stream) and 32 head blocks hand z, the skip vector and the partial logits
//     to each other as tagged granules; weights of the head stay in registers for the run
//   per step (any B): gen_wave (one workgroup per stream: PRE row (+bias), 50 × [dilated conv,
//     gate, residual] while four loader waves stream the per-layer weight images into an LDS
//     ring by LDS-DMA), gen_gemv × 3 (K-split row-vector products with deterministic partial
//     sums: skip = z_cat·SKIPcat, h = relu(relu(skip + Σb)·POST1 + b1), logits = h·POST2) and
//     gen_sample (Σ partials + b2, the draw)
// Both draw with the same wave-level inverse-CDF code: u = hash(seed, stream, step), µ-law
// decode, next input = teacher[t] or the draw (imodel.py:167-187, :260-269).
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

// ---- per-stream layer chain --------------------------------------------------------------
// One workgroup of 8 waves per stream: waves 0-3 compute (one per SIMD), waves 4-7 move data.
//   compute wave w owns channels 8w..8w+7 (lane group c = lane>>3 <-> channel 8w+c):
//     conv      lane = (c, sg = sig|gate, kq): 16 FMAs over inputs 8kq..8kq+7 of x[t-d] and of
//               x[t] (4 weight + 4 broadcast input ds_read_b128), the four lanes' sums summed
//               by two DPP quad permutes, the sig/gate partner fetched by row_half_mirror,
//               z = tanh(sig)·σ(gate) on all 8 lanes of the group
//     residual  lane = (c, kp = k-eighth): 4 FMAs over z[4kp..4kp+3], DPP-reduced over kp
//   Splitting the layer over the four SIMDs is what pays: one wave doing all 64 outputs
//   reads 43 KB of LDS per layer through one SIMD's return path (~16 cycles per 1-KiB
//   ds_read_b128), ~1,500 cycles per layer.
//   loader waves  (a) this step's dilated taps x_l[t-d_l] (ring slot t mod d_l) into the LDS tap
//                 table, two layers per 4-byte LDS-DMA; (b) every layer's slot — weights (20 ×
//                 1 KiB, packed once per gen_start) + bias rows + the stream's GC-projection
//                 row — into an NS-slot LDS ring, NS-1 layers ahead: 5 pieces + 1 row per loader
//                 per layer (counted vmcnt, inside the 6-bit counter).
// Two raw s_barriers per layer: B1 (x of layer l written; before it each loader retires layer
// l's pieces, and the compute waves' reads of slot l-1 retired, so the loaders refill it after
// B1) and B2 (z of layer l written).  No global loads on the compute chain.
// Conv lane (c, sg, kq) takes inputs 8kq..8kq+7 of BOTH taps (pieces m = 0, 1: x[t-d]; m = 2, 3:
// x[t]), so the persistent chain computes the dilated half of the next layer's conv beside the
// residual and only 8 current-tap FMAs (two chains of 4) remain between the x write and the gate
// (with the residual weights read before the z write: 36.3 -> 35.0 us per step at B = 10, same box;
// either change alone: 36.2 / 36.5)
constexpr int GI_W = 16 * 256;              // conv: [w 4][m 4][lane 64][4]  W[32(m>>1)+8kq+4(m&1)+j][32sg+8w+c]
constexpr int GI_R = 4 * 256;               // residual: [h 2][q 4][c 32][4] RES[16h+4q+j][c]
constexpr int GI_WR = GI_W + GI_R;          // 20 pieces of 1 KiB
constexpr int GIMG = GI_WR + 192;           // global image: + conv bias [64] + residual bias [64] + zeros [64]
constexpr int G_SLOT = GI_WR + 256;         // LDS slot: weights | bc [64] | br [64] | gc [64] | pad [64]
constexpr int G_NS = 6;                     // LDS ring depth (layers)
constexpr int G_PIECES = 5;                 // 1-KiB pieces per loader wave per layer (4 loaders)
constexpr int G_DMA = G_PIECES + 1;         // + one 256-B row
constexpr int G_MAXL = 256;                 // tap table rows
constexpr int G_LDS = G_NS * G_SLOT + (G_MAXL + 2) * 32 + 4 * 32 + 2 * 32;   // ring | taps | x[4 waves] | z[2]
static_assert(4 * G_PIECES * 256 == GI_WR, "image pieces");
static_assert(G_LDS * 4 <= 160 * 1024, "LDS");

struct WaveK {
  const float* pre; const float* pre_b; const float* img; const float* gc_proj;
  float* rings; float* zcat; const long long* step; const int* code;
  int B, L, nbl, Cr, Cd, pre_bias;
  long long* trace;   // non-null (LBWN_GEN_TRACE set at plan creation): stream 0's cycle stamps
};

LBWN_DEV float dot4(const floatx4& w, const floatx4& x, float acc) {
  acc = fmaf(w[0], x[0], acc);
  acc = fmaf(w[1], x[1], acc);
  acc = fmaf(w[2], x[2], acc);
  return fmaf(w[3], x[3], acc);
}

template <int CTRL>
LBWN_DEV float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141;

// workgroup barrier that retires only this wave's LDS ops: no vmcnt wait (outstanding global
// stores and LDS-DMA pieces stay in flight across it); the "memory" clobber pins LDS accesses
LBWN_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA: lane i's SIZE bytes from src land at lds_dst + i·SIZE (lds_dst wave-uniform)
LBWN_DEV void dma16(const float* src, float* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
LBWN_DEV void dma4(const float* src, float* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 4, 0, 0);
}

__global__ __launch_bounds__(512) void gen_wave_kernel(WaveK a) {
  __shared__ __attribute__((aligned(16))) float sm[G_LDS];
  float* RING = sm;                  // [G_NS][G_SLOT]
  float* XP = sm + G_NS * G_SLOT;    // [L (+2)][32] dilated taps of this step
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, b = blockIdx.x, L = a.L;
  const long t = *a.step;

  if (wid >= 4) {   // ---- loader waves
    const int lw = wid - 4;
    const float* zeros = a.img + GI_WR + 128;   // the image's zero row (layer 0)
    // (a) taps: pair q = layers 2q, 2q+1 (lane half h) by loader q % 4; d is a power of two,
    // slot = t & (d-1); ring offsets carried in scalars (no integer division)
    {
      const int h = lane >> 5, c = lane & 31;
      long roff = 0;
      int bl = 0;
      for (int q = 0; 2 * q < L; ++q) {
        const int dE = 1 << bl;
        const long roffO = roff + (long)dE * a.B * a.Cr;
        const int blO = (bl + 1 == a.nbl) ? 0 : bl + 1;
        const int dO = 1 << blO;
        if ((q & 3) == lw) {
          const int d = h ? dO : dE, l = 2 * q + h;
          const float* src = (l < L && c < a.Cr)
                                 ? a.rings + (h ? roffO : roff) + ((long)b * d + (t & (d - 1))) * a.Cr + c
                                 : zeros + c;
          dma4(src, XP + 2 * q * 32);
        }
        roff = roffO + (long)dO * a.B * a.Cr;
        bl = (blO + 1 == a.nbl) ? 0 : blO + 1;
      }
    }
    // (b) slots: pieces [5lw, 5lw+5) + row lw (bc | br | gc | pad)
    auto issue = [&](int l) {
      const float* src = a.img + (long)l * GIMG;
      float* dst = RING + (l % G_NS) * G_SLOT;
#pragma unroll
      for (int p = 0; p < G_PIECES; ++p) {
        const int pc = lw * G_PIECES + p;
        dma16(src + pc * 256 + lane * 4, dst + pc * 256);
      }
      const float* row = lw < 2 ? src + GI_WR + lw * 64
                       : lw == 2 ? (a.gc_proj ? a.gc_proj + ((long)l * a.B + b) * 64 : zeros)
                                 : zeros;
      dma4(row + lane, dst + GI_WR + lw * 64);
    };
    for (int l = 0; l < G_NS - 1 && l < L; ++l) issue(l);
    for (int k = -1; k < L; ++k) {
      // barrier k (after z_k is written; k = -1: the step input) releases the residual of layer
      // k and the conv of layer k+1, so slot k+1 must have landed.  Issued so far: taps, layers
      // 0 .. min(k+NS-2, L-1): retire all but the min(k+NS-2, L-1) - (k+1) youngest layers.
      const int younger = min(k + G_NS - 2, L - 1) - (k + 1);
      if (younger >= G_NS - 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA * (G_NS - 3)) : "memory");
      else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA * 2) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      // slot of layer k-1 is dead (its residual ran before barrier k): layer k+NS-1 goes there
      // (k = 0: the slot of layer NS-1, never used yet)
      if (k >= 0 && k + G_NS - 1 < L) issue(k + G_NS - 1);
    }
    return;
  }

  // ---- compute waves: ONE workgroup barrier per layer.  Every wave keeps the whole layer input
  // x (lane c and c+32 hold channel c) and computes the residual of all 32 channels itself
  // (16 FMAs per lane over one z half, the halves summed by v_permlane32_swap), so the next
  // layer's conv needs no second barrier: its inputs go through the wave's own LDS row (XW).
  const int w = wid, Cr = a.Cr, Cd = a.Cd;
  const int c = lane >> 3, sg = (lane >> 2) & 1, kq = lane & 3, kp = lane & 7;
  const int ch = 8 * w + c;                 // the conv channel of this lane group
  const int o = 32 * sg + ch;               // conv output of this lane
  const bool lead = kp == 0;                // one lane per group stores z
  const int rc = lane & 31, rh = lane >> 5; // residual: out channel rc over z half rh
  float* XW = XP + (G_MAXL + 2) * 32 + 32 * w;   // this wave's copy of the layer input
  float* Z = XP + (G_MAXL + 2) * 32 + 128;       // z double buffer [2][32]
  const bool tr = a.trace && b == 0 && w == 0 && lane == 0;
  if (tr) a.trace[0] = clock64();
  // step input: PRE row of the previous draw (+ PRE_BIAS); the zero vector at step 0
  float x = 0.f;    // x[rc] of the current layer input
  if (rc < Cr) {
    const int code = a.code[b];
    if (code >= 0) x = a.pre[(long)code * Cr + rc];
    if (a.pre_bias && a.pre_b) x += a.pre_b[rc];
  }
  if (lane < 32) XW[rc] = x;
  if (tr) a.trace[1] = clock64();
  long roff = 0;   // ring offset of layer l
  int bl = 0;      // l % nbl
  lds_barrier();   // barrier -1: taps and slot 0 landed, every wave's XW written
  if (tr) a.trace[2] = clock64();
  for (int l = 0; l < L; ++l) {
    const float* S = RING + (l % G_NS) * G_SLOT;
    floatx4 wv[4], xv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      wv[m] = *(const floatx4*)(S + (w * 4 + m) * 256 + lane * 4);
      xv[m] = *(const floatx4*)((m < 2 ? XP + l * 32 : XW) + 8 * kq + 4 * (m & 1));
    }
    const float bco = S[GI_WR + o] + S[GI_WR + 128 + o];
    __builtin_amdgcn_sched_barrier(0);
    const int d = 1 << bl;
    // x_l[t] into the ring (wave w stores channels 8w..8w+7)
    if (rh == 0 && (rc >> 3) == w && rc < Cr) a.rings[roff + ((long)b * d + (t & (d - 1))) * Cr + rc] = x;
    roff += (long)d * a.B * Cr;
    bl = (bl + 1 == a.nbl) ? 0 : bl + 1;
    float acc0 = dot4(wv[0], xv[0], 0.f), acc1 = dot4(wv[1], xv[1], 0.f);
    acc0 = dot4(wv[2], xv[2], acc0);
    acc1 = dot4(wv[3], xv[3], acc1);
    float v = acc0 + acc1;
    v += dpp<DPP_XOR1>(v);
    v += dpp<DPP_XOR2>(v);
    v += bco;                                      // conv output o (+ bias + GC term)
    const float vp = dpp<DPP_HALF_MIRROR>(v);      // the partner output (sig <-> gate, same channel)
    const float z = gate_z(sg ? vp : v, sg ? v : vp);
    float* Zl = Z + (l & 1) * 32;
    if (lead) {
      Zl[ch] = z;
      if (ch < Cd) a.zcat[(long)b * L * Cd + (long)l * Cd + ch] = z;
    }
    if (tr) a.trace[4 + 2 * l] = clock64();
    lds_barrier();   // barrier l: z_l complete; slot l+1 landed
    // residual of all 32 channels: x_{l+1}[rc] = x[rc] + b[rc] + Σ_k RES[k][rc]·z[k]
    floatx4 zv[4], rw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      zv[q] = *(const floatx4*)(Zl + 16 * rh + 4 * q);
      rw[q] = *(const floatx4*)(S + GI_W + ((rh * 4 + q) * 32 + rc) * 4);
    }
    const float bro = S[GI_WR + 64 + rc];
    float r0 = dot4(rw[0], zv[0], 0.f), r1 = dot4(rw[1], zv[1], 0.f);
    r0 = dot4(rw[2], zv[2], r0);
    r1 = dot4(rw[3], zv[3], r1);
    const float r = r0 + r1;
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(r), __float_as_uint(r), false, false);
    x += (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) + bro;
    if (lane < 32) XW[rc] = x;   // read back by this wave's conv of layer l+1: a wave-local sync only
    wave_sync();
    if (tr) a.trace[5 + 2 * l] = clock64();
  }
}

// per-layer weight image in the compute waves' lane order (reference layouts in, GIMG floats
// per layer out): SIGNAL/GATE [l][tap][Cr][Cd] (tap 0 = x[t-d]), RESIDUAL [l][Cd][Cr]
__global__ void gen_pack_kernel(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                const float* res, const float* res_b, float* img, int Cr, int Cd) {
  const int l = blockIdx.x;
  float* out = img + (long)l * GIMG;
  for (int e = threadIdx.x; e < GIMG; e += blockDim.x) {
    float v = 0.f;
    if (e < GI_W) {
      const int w = e / 1024, m = (e / 256) % 4, ln = (e % 256) / 4, j = e % 4;
      const int c = ln >> 3, sg = (ln >> 2) & 1, kq = ln & 3;
      const int k = (m < 2 ? 0 : 32) + 8 * kq + 4 * (m & 1) + j;
      const int tap = k >> 5, in = k & 31, oc = 8 * w + c;
      if (in < Cr && oc < Cd) v = (sg ? gate : sig)[(long)l * 2 * Cr * Cd + (tap * Cr + in) * Cd + oc];
    } else if (e < GI_WR) {
      const int f = e - GI_W, j = f & 3, oc = (f >> 2) & 31, q = (f >> 7) & 3, h = f >> 9;
      const int zc = 16 * h + 4 * q + j;
      if (zc < Cd && oc < Cr) v = res[(long)l * Cd * Cr + zc * Cr + oc];
    } else {
      const int f = e - GI_WR;
      if (f < 64) {
        const float* bb = f < 32 ? sig_b : gate_b;
        if (bb && (f & 31) < Cd) v = bb[(long)l * Cd + (f & 31)];
      } else if (f < 128) {
        if (res_b && f - 64 < Cr) v = res_b[(long)l * Cr + f - 64];
      }
    }
    out[e] = v;
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
  long long* step_advance;                      // non-null: block (0,0) advances the step counter
  long long* trace;                             // debug (LBWN_GEN_TRACE): [8] stamps of this launch
};

__global__ __launch_bounds__(256) void gen_gemv_kernel(GemvK a) {
  // staged inputs per wave: xs[w][i][j] = x[j][k0 + w + 4i], so a wave reads the 16 stream
  // values of one of its rows with 4 broadcast ds_read_b128 (not 16 ds_read_b32)
  __shared__ __attribute__((aligned(16))) float xs[4][GV_KSL_MAX / 4][16];
  __shared__ float red[4][16][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int KSL = a.KSL, ks = blockIdx.y, k0 = ks * KSL, k1 = min(a.K, k0 + KSL);
  const bool first = blockIdx.x == 0 && blockIdx.y == 0, last = blockIdx.x == gridDim.x - 1 && blockIdx.y == gridDim.y - 1;
  if (a.trace && tid == 0 && first) { a.trace[0] = wall_clock64(); a.trace[2] = clock64(); }
  if (a.trace && tid == 0 && last) a.trace[6] = wall_clock64();
  // weights: branch-free (clamped index, then select), so hipcc can count these loads and the
  // input staging below does not wait for them (behind branches it lost the count and waited
  // vmcnt(0): the weight fetch and the input fetch became two serial round trips)
  float wr[GV_KSL_MAX / 4];
#pragma unroll
  for (int i = 0; i < GV_KSL_MAX / 4; ++i) {
    const int k = k0 + w + 4 * i;
    wr[i] = a.W[(long)min(k, a.K - 1) * a.ldw + min(n, a.N - 1)];
    if (!(4 * i < KSL && k < k1 && n < a.N)) wr[i] = 0.f;
  }
  if (a.step_advance && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0)   // no-return atomic: no wait
    __hip_atomic_fetch_add(a.step_advance, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto put = [&](int e, float x) {   // element e = j·KSL + kk of the slice
    const int j = e / KSL, kk = e % KSL;
    xs[kk & 3][kk >> 2][j] = x;
  };
  for (int b0 = 0; b0 < a.B; b0 += 16) {
    const int nbb = min(16, a.B - b0);
    // stage the input slice: every load of this thread issued before the first is consumed
    constexpr int GV_EPT = 16 * GV_KSL_MAX / 256;
    if (a.in_part) {
      // the previous GEMV's partials (≤ 32 per element, all issued at once: one memory round
      // trip) + bias, relu; two elements per pass
      for (int r0 = 0; r0 < GV_EPT; r0 += 2) {
        if (tid + 256 * r0 >= 16 * KSL) break;
        float s2[2] = {0.f, 0.f}, bb[2];
        for (int q0 = 0; q0 < a.in_parts; q0 += 32) {
          float v[2][32];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = tid + 256 * (r0 + h), j = min(e / KSL, nbb - 1), k = min(k0 + e % KSL, a.K - 1);
            const float* pp = a.in_part + (long)(b0 + j) * a.K + k;
#pragma unroll
            for (int i = 0; i < 32; ++i) v[h][i] = pp[(long)min(q0 + i, a.in_parts - 1) * a.B * a.K];
            if (q0 == 0) bb[h] = a.in_bias ? a.in_bias[k] : 0.f;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 32; ++i) s2[h] += (q0 + i < a.in_parts) ? v[h][i] : 0.f;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = tid + 256 * (r0 + h);
          if (e >= 16 * KSL) continue;
          const int j = e / KSL, k = k0 + e % KSL;
          float v = 0.f;
          if (j < nbb && k < a.K) {
            v = s2[h] + bb[h];
            if (a.relu_in) v = fmaxf(v, 0.f);
          }
          put(e, v);
        }
      }
    } else {
      float v[GV_EPT];
#pragma unroll
      for (int r = 0; r < GV_EPT; ++r) {
        const int e = tid + 256 * r, j = min(e / KSL, nbb - 1), k = min(k0 + e % KSL, a.K - 1);
        v[r] = a.in[(long)(b0 + j) * a.ldin + k];
      }
#pragma unroll
      for (int r = 0; r < GV_EPT; ++r) {
        const int e = tid + 256 * r;
        if (e >= 16 * KSL) continue;
        const int j = e / KSL, kk = e % KSL;
        float x = (j < nbb && k0 + kk < a.K) ? v[r] : 0.f;
        if (a.relu_in) x = fmaxf(x, 0.f);
        put(e, x);
      }
    }
    __syncthreads();
    if (a.trace && tid == 0 && first && b0 == 0) a.trace[3] = clock64();
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
    for (int i = 0; i < GV_KSL_MAX / 4; ++i)
      if (4 * i < KSL) {
        const floatx4* xr = (const floatx4*)&xs[w][i][0];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 x = xr[q];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[4 * q + jj] = fmaf(x[jj], wr[i], acc[4 * q + jj]);
        }
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
  if (a.trace && tid == 0 && first) { a.trace[4] = clock64(); a.trace[1] = wall_clock64(); }
  if (a.trace && tid == 0 && last) a.trace[7] = wall_clock64();
}

// ---- the draw (imodel.py:167-187, :260-269) ----------------------------------------------
// Inverse-CDF draw of softmax(logits): the first k with cumsum(e)[k] > u·Σe, e = exp(logits -
// max), u = hash(seed, stream, step) (oracle/wavenet_ref.py sample_from_logits restates the
// transform).  Wave-level only — lane = a contiguous run of ceil(Q/64) codes, shuffles, no
// workgroup barrier — so every wave that calls it with the same logits draws the same code.
struct DrawK {
  const float* part; int parts; const float* bias;   // logits = Σ part[p][b][:] + bias (per-step path)
  int Q, B;
  float* logits; int* samples; float* wav; long long max_steps;
  const int* teacher; long long n_teacher; unsigned long long seed; int* code;
};

// wave-wide max / min / inclusive scan on DPP (row ops + row_bcast, GFX9): one VALU latency
// per step instead of a ds_bpermute round trip per __shfl step
template <int CTRL, int ROWS = 0xF>
LBWN_DEV int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, true); }
LBWN_DEV float wave_max(float v) {
  v = fmaxf(v, __int_as_float(dpp_i<0xB1>(__float_as_int(v))));    // quad_perm xor 1
  v = fmaxf(v, __int_as_float(dpp_i<0x4E>(__float_as_int(v))));    // quad_perm xor 2
  v = fmaxf(v, __int_as_float(dpp_i<0x141>(__float_as_int(v))));   // row_half_mirror
  v = fmaxf(v, __int_as_float(dpp_i<0x140>(__float_as_int(v))));   // row_mirror: every row uniform
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
// inclusive prefix sum over the 64 lanes: Hillis-Steele within rows (row_shr 1, 2, 4, 8), then
// row 15's total into rows 1, 3 and lane 31's into rows 2, 3
LBWN_DEV float wave_scan(float x) {
  x += __int_as_float(dpp_i<0x111>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x112>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x114>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x118>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x142, 0xA>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x143, 0xC>(__float_as_int(x)));
  return x;
}

LBWN_DEV uint64_t splitmix(uint64_t seed, uint64_t stream, uint64_t step) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ULL + (stream << 32) + step + 0x632BE59BD9B4E019ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// v[j] = logit of code lane·per + j.  Returns the next input code of stream b after step t (the
// teacher's or the draw); the writing wave stores logits, the sample, its µ-law decode, code[b].
// µ-law decode of one code (ops.py:12-20)
LBWN_DEV float mu_decode_q(int q, int Q) {
  const float mu = (float)(Q - 1), inv = 1.f / mu;
  const float aa = (2.f * (float)q - 1.f) * inv - 1.f;
  const float sg = aa > 0.f ? 1.f : (aa < 0.f ? -1.f : 0.f);
  return sg * (powf(1.f + mu, fabsf(aa)) - 1.f) * inv;
}

// the persistent form's wav: its draws store only the code (powf on lane 0 held the next step's
// PRE row behind it); this decodes the run's samples [step - n, step) after the launch
__global__ void gen_decode_kernel(const int* __restrict__ samples, float* __restrict__ wav, const long long* step,
                                  int B, long long max_steps, int n, int Q) {
  const long long t1 = min(*step, max_steps), t0 = max(*step - n, 0LL);
  const long long span = t1 - t0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * span;
       e += (long long)gridDim.x * blockDim.x) {
    const long long i = (e / span) * max_steps + t0 + e % span;
    wav[i] = mu_decode_q(samples[i], Q);
  }
}

template <int MP>
LBWN_DEV int draw_core(float (&v)[MP], const DrawK& a, int b, long long t, bool write, bool decode = true) {
  const int lane = threadIdx.x & 63, Q = a.Q;
  const int per = (Q + 63) >> 6, c0 = lane * per;
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    const bool ok = j < per && c0 + j < Q;
    if (ok) mx = fmaxf(mx, v[j]);
    if (ok && write) a.logits[(long)b * Q + c0 + j] = v[j];
  }
  mx = wave_max(mx);
  float e[MP], loc = 0.f;
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    e[j] = (j < per && c0 + j < Q) ? expf(v[j] - mx) : 0.f;
    loc += e[j];
  }
  const float incl = wave_scan(loc);
  const float total = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
  const float excl = incl - loc;
  const uint64_t h = splitmix(a.seed, (uint64_t)b, (uint64_t)t);
  const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
  const float target = u * total;
  int found = Q;   // the lane whose run contains the crossing point
  if (excl <= target && target < incl) {
    float run = excl;
#pragma unroll
    for (int j = 0; j < MP; ++j) {
      if (j < per && c0 + j < Q && found == Q) {
        run += e[j];
        if (run > target) found = c0 + j;
      }
    }
    if (found == Q) found = min(c0 + per, Q) - 1;
  }
  found = wave_min(found);
  if (found >= Q) found = Q - 1;
  const int next = (t < a.n_teacher) ? a.teacher[t] : found;   // imodel.py:260-269
  if (write && lane == 0) {
    if (t < a.max_steps) {
      a.samples[(long)b * a.max_steps + t] = found;
      if (decode) a.wav[(long)b * a.max_steps + t] = mu_decode_q(found, Q);
    }
    a.code[b] = next;
  }
  return next;
}

// per-step path: logits from the post2 GEMV's K-slice partials, Σ in slice order + bias
template <int MP>
LBWN_DEV int draw_wave(const DrawK& a, int b, long long t, bool write) {
  const int lane = threadIdx.x & 63, Q = a.Q;
  const int per = (Q + 63) >> 6, c0 = lane * per;
  float v[MP], bv[MP];
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    v[j] = 0.f;
    bv[j] = a.bias ? a.bias[min(c0 + j, Q - 1)] : 0.f;
  }
  constexpr int CH = MP > 4 ? 8 : 16;
  for (int q0 = 0; q0 < a.parts; q0 += CH) {   // every load of a chunk (and the bias) issued before the first add
    float x[MP][CH];
#pragma unroll
    for (int j = 0; j < MP; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i)
        x[j][i] = a.part[((long)min(q0 + i, a.parts - 1) * a.B + b) * Q + min(c0 + j, Q - 1)];
#pragma unroll
    for (int j = 0; j < MP; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i) v[j] += (q0 + i < a.parts) ? x[j][i] : 0.f;
  }
  if (a.bias) {
#pragma unroll
    for (int j = 0; j < MP; ++j) v[j] += bv[j];
  }
  return draw_core<MP>(v, a, b, t, write);
}

// the per-step path's sampler: one wave per stream; the step counter was advanced by this
// step's skip GEMV, so this step is *step - 1
__global__ __launch_bounds__(64) void gen_sample_kernel(DrawK a, const long long* step) {
  const long long t = *step - 1;
  if (a.Q > 256) draw_wave<8>(a, blockIdx.x, t, true);
  else draw_wave<4>(a, blockIdx.x, t, true);
}

#ifndef LBWN_GEN_SUBSTAMPS
#define LBWN_GEN_SUBSTAMPS 0
#endif
constexpr long long G_SPIN_TIMEOUT = 400000000LL;   // wall_clock64 ticks (100 MHz) = 4 s

// ---- persistent generation: one launch per run (stream groups of <= 16) ----------------
// Roles (one 512-thread workgroup per CU, all resident): streams split into groups of Bg <= 16, each
// group's Bg chain blocks and P_NH head blocks hand off among themselves only (groups x (Bg + P_NH)
// <= CUs; B = 64: four groups, 192 blocks); within a group:
//   chain block b < B   per step: draw the previous step (gather the P_NH partial-logit
//                       granules of stream b, Σ + b2, wave-level draw), PRE row, 50 layers as in
//                       gen_wave (LDS-DMA ring continuous across steps; the next step's taps are
//                       DMA'd right after the last layer), z_l published as tagged granules
//   head block m < P_NH owns skip columns [16m, 16m+16), post1 columns [16m, 16m+16) and the
//                       same post2 rows (POST1 / POST2 slices held in registers for the run):
//                       A. accumulates its skip columns layer by layer as the z granules arrive
//                          (SKIP slice streamed from L2 one layer ahead);
//                       B. publishes them, gathers the whole skip vector, relu(· + Σb);
//                       C. h = relu(skip·POST1[:, cols] + b1), partial logits h·POST2[rows, :]
//                          published as granules for the chain blocks' draw.
// Every hand-off is an 8-byte {value, tag = step + 1} granule written by one sc1 store and polled
// with relaxed agent-scope loads (no flag, no fence: MI355X_MICROARCH.md § visibility, R2);
// single-buffered, because no producer can run a step ahead of its slowest consumer (each
// stage waits on the previous one through the whole ring of roles).  Every spin is bounded
// (status 5).  Three hops per step (z tail, skip all-gather, logit partials) replace the
// per-step path's four launch boundaries and its weight re-fetches.
constexpr int P_NH = 32;     // head blocks
constexpr int P_MAXB = 16;   // streams per group (phase A maps 16 columns x 16 streams onto 512 threads)
constexpr int P_MAXL = 236;  // layers (the draw's two half-sums use tap-table rows 240..255)
constexpr int P_DLROW = 240;
constexpr int P_LA = 8;      // layers per head round (phase A)

struct PersistK {
  const float* pre; const float* pre_b; const float* img; const float* gc_proj;
  float* rings; long long* step; const int* code_in;
  int B, L, nbl, Cr, Cd, pre_bias, n_steps;
  unsigned long long* zg;   // [B][L][32] z granules
  int Cs, Cp, Q;
  const float* skipw; const float* bsum; const float* post1; const float* post1_b; const float* post2;
  unsigned long long* sg;   // [B][Cs] skip granules
  unsigned long long* lg;   // [P_NH][B][Q] partial-logit granules
  DrawK draw;               // outputs; draw.bias = b2
  int* status;
  long long* trace;         // wall stamps of the run's last step (tools/gen_trace.py), or null
  int Bg;                   // streams per group: block g·(Bg + P_NH) + r is group g's chain block r < Bg
                            // (stream g·Bg + r) or head block r - Bg; groups hand off only inside
  long long* gstep;         // step counters of groups 1.. (group 0's is *step, the plan's "step")
};

// poll granules base[off + i·stride], i < nv (N at most; the rest re-read granule nv-1), until
// every tag matches; v[i] = payload.  base is wave-uniform and the index 32-bit, so each load
// is one VGPR offset on an SGPR base.  After any timeout (status != 0) every sweep gives up at
// once, so a failed hand-off drains the launch instead of waiting out each later spin.
template <int N>
LBWN_DEV void sweep(const unsigned long long* base, unsigned off, unsigned stride, int nv, unsigned tag, float (&v)[N],
                    int* status) {
  long long ts = 0;
  const unsigned last = (unsigned)max(nv - 1, 0);
  for (unsigned spins = 1;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const unsigned idx = off + min((unsigned)i, last) * stride;
      const unsigned long long x = __hip_atomic_load(base + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[i] = __uint_as_float((unsigned)x);
      ok &= (unsigned)(x >> 32) == tag;
    }
    if (ok) return;
    if ((spins & 31) == 0) {   // the clock and the status word cost a round trip each: not every retry
      if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
      const long long now = wall_clock64();
      if (ts == 0) ts = now;
      else if (now - ts > G_SPIN_TIMEOUT) {
        __hip_atomic_store(status, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

LBWN_DEV void put_granule(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// ring slot DMA with sc1 (L2-served): a tap line this CU read d steps ago may still sit in its L1
LBWN_DEV void dma4_sc1(const float* src, float* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 4, 0, 16);
}


LBWN_DEV void persist_chain(const PersistK& a, float* sm, int b, long long* stepc, long long* trace) {
  float* RING = sm;                  // [G_NS][G_SLOT]
  float* XP = sm + G_NS * G_SLOT;    // [L][32] dilated taps of this step
  float* DL = XP + P_DLROW * 32;     // [2][256] half-sums of the partial logits of the step being drawn
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, L = a.L, n = a.n_steps;
  const long long t0 = *stepc;
  const long GT = (long)n * L;       // layers of the run, in order: global index g = s·L + l

  if (wid >= 4) {   // ---- loader waves
    const int lw = wid - 4;
    const float* zeros = a.img + GI_WR + 128;
    auto taps = [&](long long t) {   // as gen_wave (a), for step t
      const int h = lane >> 5, c = lane & 31;
      long roff = 0;
      int bl = 0;
      for (int q = 0; 2 * q < L; ++q) {
        const int dE = 1 << bl;
        const long roffO = roff + (long)dE * a.B * a.Cr;
        const int blO = (bl + 1 == a.nbl) ? 0 : bl + 1;
        const int dO = 1 << blO;
        if ((q & 3) == lw) {
          const int d = h ? dO : dE, l = 2 * q + h;
          const float* src = (l < L && c < a.Cr)
                                 ? a.rings + (h ? roffO : roff) + ((long)b * d + (t & (d - 1))) * a.Cr + c
                                 : zeros + c;
          dma4_sc1(src, XP + 2 * q * 32);
        }
        roff = roffO + (long)dO * a.B * a.Cr;
        bl = (blO + 1 == a.nbl) ? 0 : blO + 1;
      }
    };
    // the layer and ring slot of the next issue, advanced with wrap-around: g mod L and g mod G_NS
    // of a 64-bit g were two long divisions per layer on the loaders' path to every barrier
    int iss_l = 0, iss_slot = 0;
    auto issue = [&](long /*g: layer iss_l, slot iss_slot*/) {   // weights of global layer g into slot g mod G_NS
      const int l = iss_l;
      const float* src = a.img + (long)l * GIMG;
      float* dst = RING + iss_slot * G_SLOT;
      iss_l = (iss_l + 1 == L) ? 0 : iss_l + 1;
      iss_slot = (iss_slot + 1 == G_NS) ? 0 : iss_slot + 1;
#pragma unroll
      for (int p = 0; p < G_PIECES; ++p) {
        const int pc = lw * G_PIECES + p;
        dma16(src + pc * 256 + lane * 4, dst + pc * 256);
      }
      const float* row = lw < 2 ? src + GI_WR + lw * 64
                       : lw == 2 ? (a.gc_proj ? a.gc_proj + ((long)l * a.B + b) * 64 : zeros)
                                 : zeros;
      dma4(row + lane, dst + GI_WR + lw * 64);
    };
    taps(t0);
    long issued = 0;
    for (; issued < G_NS - 1 && issued < GT; ++issued) issue(issued);
    auto gather_half = [&](long long t) {   // partial logits of heads 16..31 for code q
      const int q = min((int)threadIdx.x - 256, a.Q - 1);
      float v[P_NH / 2], sum = 0.f;
      sweep<P_NH / 2>(a.lg, (unsigned)(((P_NH / 2) * a.B + b) * a.Q + q), (unsigned)(a.B * a.Q), P_NH / 2, (unsigned)t,
                      v, a.status);
#pragma unroll
      for (int i = 0; i < P_NH / 2; ++i) sum += v[i];
      DL[256 + q] = sum;
    };
    for (int s = 0; s < n; ++s) {
      if (s > 0) {
        gather_half(t0 + s);
        lds_barrier();   // D: the previous step's logits are in DL
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();              // -1: taps and the first slot landed, every wave's XW written
      for (int k = 0; k < L; ++k) {
        const long G = (long)s * L + k;
        // barrier G releases the residual of layer G and the conv of G+1: retire all but the
        // slots younger than G+1
        const long younger = (issued - 1) - (G + 1);
        if (younger >= G_NS - 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA * (G_NS - 3)) : "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA * 2) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_DMA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (issued < GT) issue(issued++);   // into the slot of layer G-1 (dead after barrier G)
        if (k == L - 1 && s + 1 < n) taps(t0 + s + 1);   // the ring stores of step s landed (compute waves drained)
      }
    }
    gather_half(t0 + n);
    lds_barrier();   // D of the run's last draw
    return;
  }

  // ---- compute waves
  const int w = wid, Cr = a.Cr, Cd = a.Cd;
  const int c = lane >> 3, sg = (lane >> 2) & 1, kq = lane & 3, kp = lane & 7;
  const int ch = 8 * w + c, o = 32 * sg + ch;
  const bool lead = kp == 0;
  const int rc = lane & 31, rh = lane >> 5;
  float* XW = XP + (G_MAXL + 2) * 32 + 32 * w;
  float* Z = XP + (G_MAXL + 2) * 32 + 128;
  const int Q = a.Q, per = (Q + 63) >> 6, c0 = lane * per;
  long long* tr = (trace && b == 0 && threadIdx.x == 0) ? trace : nullptr;
  float bq[4];               // b2 of this lane's codes, loaded once (a global load in every draw before)
#pragma unroll
  for (int j = 0; j < 4; ++j) bq[j] = a.draw.bias ? a.draw.bias[min(c0 + j, Q - 1)] : 0.f;
  int code = a.code_in[b];   // step 0 of the run: the previous run's last draw (-1 at t = 0)
  float accd = 0.f;          // the dilated-tap partial of the next layer's conv
  auto dilated = [&](const float* Sl, int l) {
    const floatx4 w0 = *(const floatx4*)(Sl + (w * 4) * 256 + lane * 4);
    const floatx4 w1 = *(const floatx4*)(Sl + (w * 4 + 1) * 256 + lane * 4);
    const floatx4 x0 = *(const floatx4*)(XP + l * 32 + 8 * kq), x1 = *(const floatx4*)(XP + l * 32 + 8 * kq + 4);
    return dot4(w1, x1, dot4(w0, x0, 0.f));
  };
  int slot = 0;              // ring slot of global layer G = s·L + l (G mod G_NS, advanced per layer)
  for (int s = 0; s <= n; ++s) {
    const long long t = t0 + s;
    if (s > 0) {
      // draw step t-1: code q's partial logits of heads 0..15 here, 16..31 by the loader waves;
      // logit = (Σ first half + Σ second half) + b2
      const int q = min((int)threadIdx.x, Q - 1);
      float v[P_NH / 2], lsum = 0.f;
      sweep<P_NH / 2>(a.lg, (unsigned)(b * Q + q), (unsigned)(a.B * Q), P_NH / 2, (unsigned)t, v, a.status);
#pragma unroll
      for (int i = 0; i < P_NH / 2; ++i) lsum += v[i];
      DL[q] = lsum;
      if (tr && s == n) tr[5] = wall_clock64();
      lds_barrier();   // D
      if (tr && s == n) tr[7] = wall_clock64();
      float lv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cc = min(c0 + j, Q - 1);
        lv[j] = DL[cc] + DL[256 + cc];
        if (a.draw.bias) lv[j] += bq[j];
      }
      code = draw_core<4>(lv, a.draw, b, t - 1, w == 0, false);
      if (s == n) {
        if (tr) tr[6] = wall_clock64();
        break;
      }
    }
    if (tr && s == n - 1) tr[0] = wall_clock64();
    float x = 0.f;   // x[rc] of the current layer input: PRE row of the draw (+ PRE_BIAS); zero at t = 0
    if (rc < Cr) {
      if (code >= 0) x = a.pre[(long)code * Cr + rc];
      if (a.pre_bias && a.pre_b) x += a.pre_b[rc];
    }
    if (lane < 32) XW[rc] = x;
    long roff = 0;
    int bl = 0;
    lds_barrier();   // -1
    accd = dilated(RING + slot * G_SLOT, 0);   // this step's taps and layer 0's slot landed by -1
    for (int l = 0; l < L; ++l) {
      const float* S = RING + slot * G_SLOT;
      slot = (slot + 1 == G_NS) ? 0 : slot + 1;
      floatx4 wv[2], xv[2];   // the current tap's pieces; the dilated half is in accd
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        wv[mm] = *(const floatx4*)(S + (w * 4 + 2 + mm) * 256 + lane * 4);
        xv[mm] = *(const floatx4*)(XW + 8 * kq + 4 * mm);
      }
      const float bco = S[GI_WR + o] + S[GI_WR + 128 + o];
      // (round 2: reading ALL of layer l+1's conv operands right after barrier l, and this layer's
      // residual weights ahead of the conv, measured 38.0 -> 38.9 us per step; what is kept is
      // the dilated half after the barrier and the residual weights just before the z write)
      // sub-layer cycle stamps (trace only): layers 16..23 of the traced step, 6 per layer
      // (compiled in only with -DLBWN_GEN_SUBSTAMPS=1: the lane-divergent stamp branches split the
      // layer into basic blocks the scheduler cannot overlap, 38.5 -> 44 us per step at B = 10)
      long long* st6 = (LBWN_GEN_SUBSTAMPS && tr && s == n - 1 && l >= 16 && l < 24 && L + 184 <= 2 * L + 136)
                           ? tr + 8 + L + 128 + 6 * (l - 16) : nullptr;
      if (st6) st6[0] = clock64();
      __builtin_amdgcn_sched_barrier(0);
      const int d = 1 << bl;
      if (rh == 0 && (rc >> 3) == w && rc < Cr) a.rings[roff + ((long)b * d + (t & (d - 1))) * Cr + rc] = x;
      roff += (long)d * a.B * Cr;
      bl = (bl + 1 == a.nbl) ? 0 : bl + 1;
      const float acc0 = dot4(wv[0], xv[0], accd), acc1 = dot4(wv[1], xv[1], 0.f);
      float v = acc0 + acc1;
      v += dpp<DPP_XOR1>(v);
      v += dpp<DPP_XOR2>(v);
      v += bco;
      if (st6) { asm volatile("" ::"v"(v)); st6[1] = clock64(); }
      const float vp = dpp<DPP_HALF_MIRROR>(v);
      const float z = gate_z(sg ? vp : v, sg ? v : vp);
      if (st6) { asm volatile("" ::"v"(z)); st6[2] = clock64(); }
      float* Zl = Z + (l & 1) * 32;
      // residual weights (slot resident since the last barrier) issued before the z write: the
      // barrier's lgkmcnt(0) retires them together with it, so only z is read after the barrier
      floatx4 rw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) rw[q] = *(const floatx4*)(S + GI_W + ((rh * 4 + q) * 32 + rc) * 4);
      const float bro = S[GI_WR + 64 + rc];
      if (lead) {
        Zl[ch] = z;
        if (ch < Cd) put_granule(a.zg + ((long)b * L + l) * 32 + ch, (unsigned)(t + 1), z);
      }
      // the last layer's ring stores must land before the loaders DMA the next step's taps
      if (l == L - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      if (st6) st6[3] = clock64();
      accd = dilated(RING + slot * G_SLOT, min(l + 1, L - 1));   // layer l+1's slot landed by this barrier
      floatx4 zv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) zv[q] = *(const floatx4*)(Zl + 16 * rh + 4 * q);
      float r0 = dot4(rw[0], zv[0], 0.f), r1 = dot4(rw[1], zv[1], 0.f);
      r0 = dot4(rw[2], zv[2], r0);
      r1 = dot4(rw[3], zv[3], r1);
      const float r = r0 + r1;
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(r), __float_as_uint(r), false, false);
      x += (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) + bro;
      if (st6) { asm volatile("" ::"v"(x)); st6[4] = clock64(); }
      if (lane < 32) XW[rc] = x;
      wave_sync();
      if (st6) st6[5] = clock64();
      if (tr && s == n - 1) tr[8 + l] = wall_clock64();
    }
    if (tr && s == n - 1) tr[1] = wall_clock64();
  }
  if (b % a.Bg == 0 && threadIdx.x == 0) *stepc = t0 + n;   // the group's blocks read it at their start
}

// the head's LDS carve (below) within the kernel's static allocation, at the largest Q (256)
static_assert(2 * P_LA * 528 + P_MAXB * 516 + 32 * 256 + 272 + 16 * 516 + 16 * 256 <= G_LDS, "head LDS");

LBWN_DEV void persist_head(const PersistK& a, int m, float* sm, int b0, int B, long long* stepc, long long* trace) {
  // B: this group's streams b0 .. b0+B-1 (granule and logit layouts are over all a.B streams)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int L = a.L, Cd = a.Cd, Cs = a.Cs, Cp = a.Cp, Q = a.Q, n = a.n_steps;
  const long long t0 = *stepc;
  // row paddings (33, 516, 17 floats) put the 16 stream rows a 16-lane MFMA operand read touches
  // on distinct banks (unpadded, the 32- / 512- / 16-float rows were 8- to 16-way conflicts)
  float* ZS = sm;                  // [2][P_LA layers][16 b][33] z of a round (double-buffered)
  float* RS = ZS + 2 * P_LA * 528; // [16 b][516] relu(skip + Σb), zero-padded
  float* HP = RS + P_MAXB * 516;   // [8 waves][64 lanes][4] MFMA partials (skip, then post1)
  float* HS = HP + 32 * 256;       // [16 b][17] h
  float* P1T = HS + 272;           // [16 c][516] POST1[:, 16m + c] (rows padded: conflict-free b128 reads)
  float* P2S = P1T + 16 * 516;     // [16 r][Q] POST2[16m + r, :]
  for (int e = tid; e < P_MAXB * 516; e += 512) RS[e] = 0.f;
  for (int e = tid; e < 16 * 512; e += 512) {   // the head's weight slices stay in LDS for the run
    const int cc = e >> 9, k = e & 511;
    P1T[cc * 516 + k] = (k < Cs && m * 16 + cc < Cp) ? a.post1[(long)k * Cp + m * 16 + cc] : 0.f;
  }
  for (int e = tid; e < 16 * Q; e += 512) {
    const int r = e / Q, q = e - r * Q;
    P2S[e] = (m * 16 + r < Cp) ? a.post2[(long)(m * 16 + r) * Q + q] : 0.f;
  }
  // lane roles: c = column within this block's 16, kg = tid >> 4 = 4·wave + (lane >> 4)
  const int c = tid & 15, kg = tid >> 4, kql = lane >> 4;
  const int scol = m * 16 + c, hcol = m * 16 + c, scol16 = m * 16;
  // A: wave wv takes layer l0 + wv of each round, lane quarter kql the channels 8kql..8kql+7
  const float* wsrc = a.skipw + (long)(8 * kql) * Cs + min(scol, Cs - 1);
  // C: post1 rows 16kg .. 16kg+15 of column hcol (P1T); post2 rows 16m .. 16m+15 of column tid (P2S)
  const float b1 = (hcol < Cp && a.post1_b) ? a.post1_b[hcol] : 0.f;
  // z granules polled by this thread: (stream zb0, channel zk) of every layer of a round
  const int zb0 = tid >> 5, zk = tid & 31;
  const bool zn0 = zb0 < B && zk < Cd;
  long long* tr = (trace && m == P_NH - 1 && tid == 0) ? trace : nullptr;
  for (int s = 0; s < n; ++s) {
    const unsigned tag = (unsigned)(t0 + s + 1);
    // A. skip columns, P_LA layers per round: the round's z granules (thread: stream tid >> 5,
    //    channel tid & 31, every layer of the round) and this lane's 8 weights arrive in one round
    //    trip; wave wv accumulates layer l0 + wv of each round into a 16x16 (stream x column)
    //    tile on v_mfma_f32_16x16x4_f32 (8 MFMAs over the layer's 32 channels: A[i = stream][k] =
    //    z, B[k][j = column] = SKIP), summed over the waves once after the last round.  (Round 3's
    //    per-thread FMAs re-read every z row for all 16 columns: ~260 KB of LDS per round.)
    floatx4 pacc = {0.f, 0.f, 0.f, 0.f};
    // rounds are aligned to the END of the stack: the last round is layer L-1 alone, so the
    // round before it finishes while the chains run their last layer and the tail after the
    // chains is one poll + one layer (the first round takes the remainder)
    const int first = (L - 1) % P_LA == 0 ? P_LA : (L - 1) % P_LA;
    const int i16 = lane & 15, kk = lane >> 4;
    for (int l0 = 0, r = 0; l0 < L; l0 += (l0 == 0 ? first : P_LA), ++r) {
      const int nl = l0 == L - 1 ? 1 : (l0 == 0 ? min(first, L) : P_LA), li = l0 + wv;
      float w8[8], zv[P_LA];
      const float* wl = a.skipw + (long)min(li, L - 1) * Cd * Cs + min(scol16 + i16, Cs - 1);
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) w8[s4] = wl[(long)min(4 * s4 + kk, Cd - 1) * Cs];
      sweep<P_LA>(a.zg, (unsigned)((b0 + (zn0 ? zb0 : 0)) * L + l0) * 32 + (zn0 ? zk : 0), 32u, nl, tag, zv, a.status);
      if (tr && s == n - 1) tr[8 + L + 40 + r] = wall_clock64();
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4)
        if (li >= L || 4 * s4 + kk >= Cd || scol16 + i16 >= Cs) w8[s4] = 0.f;
      float* Z = ZS + (r & 1) * (P_LA * 528);   // the other buffer's readers finished last round
#pragma unroll
      for (int i = 0; i < P_LA; ++i) Z[i * 528 + zb0 * 33 + zk] = (zn0 && i < nl) ? zv[i] : 0.f;
      __syncthreads();
      if (tr && s == n - 1) tr[8 + L + 80 + r] = wall_clock64();
      const float* zr = Z + wv * 528 + i16 * 33 + kk;
      float za[8];
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) za[s4] = zr[4 * s4];
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) pacc = __builtin_amdgcn_mfma_f32_16x16x4f32(za[s4], w8[s4], pacc, 0, 0, 0);
      if (tr && s == n - 1) tr[8 + L + r] = wall_clock64();
    }
    // the eight waves' tiles summed through LDS in a fixed order; thread (lane l, e): stream
    // 4(l >> 4) + e, column l & 15
    *(floatx4*)(HP + (wv * 64 + lane) * 4) = pacc;
    __syncthreads();
    if (tid < 256) {
      const int l = tid & 63, e = tid >> 6, sb = 4 * (l >> 4) + e, cc = l & 15;
      float v[8], x = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v[g] = HP[(g * 64 + l) * 4 + e];
#pragma unroll
      for (int g = 0; g < 8; ++g) x += v[g];
      if (sb < B && scol16 + cc < Cs) put_granule(a.sg + (long)(b0 + sb) * Cs + scol16 + cc, tag, x);   // B. publish
    }
    if (tr && s == n - 1) tr[2] = wall_clock64();
    // every head's own stamps (trace only): skip columns published, whole skip vector gathered
    long long* th = (trace && tid == 0 && s == n - 1) ? trace + 2 * L + 136 + 2 * m : nullptr;
    if (th) th[0] = wall_clock64();
    // B. gather the whole skip vector: thread k = tid polls column k of every stream
    if (tid < Cs) {
      // as many granule loads per poll as the group has streams, in fours (a group of 10 polled
      // 16 per thread before: 6 re-reads of its last stream)
      float v[P_MAXB];
      const unsigned o0 = (unsigned)(b0 * Cs + tid);
      if (B <= 4) sweep<4>(a.sg, o0, (unsigned)Cs, B, tag, *reinterpret_cast<float(*)[4]>(v), a.status);
      else if (B <= 8) sweep<8>(a.sg, o0, (unsigned)Cs, B, tag, *reinterpret_cast<float(*)[8]>(v), a.status);
      else if (B <= 12) sweep<12>(a.sg, o0, (unsigned)Cs, B, tag, *reinterpret_cast<float(*)[12]>(v), a.status);
      else sweep<P_MAXB>(a.sg, o0, (unsigned)Cs, B, tag, v, a.status);
      const float bs = a.bsum ? a.bsum[tid] : 0.f;
#pragma unroll
      for (int bb = 0; bb < P_MAXB; ++bb)
        if (bb < B) RS[bb * 516 + tid] = fmaxf(v[bb] + bs, 0.f);
    }
    __syncthreads();
    if (tr && s == n - 1) tr[3] = wall_clock64();
    if (th) th[1] = wall_clock64();
    // C. h = relu(relu(skip + Σb)·POST1[:, cols] + b1) for this block's 16 columns and all 16
    //    stream slots on v_mfma_f32_16x16x4_f32 (exact f32 products): wave wv takes K rows
    //    64wv .. 64wv+63 (16 MFMAs; A[i = stream][k] = RS, B[k][j = column] = P1T), the eight
    //    16x16 partials are summed through LDS in a fixed order.  (Round 3's per-thread FMA form
    //    re-read each RS row for all 16 columns: ~390 KB of LDS reads, ~1.1 us.)
    {
      const int i16 = lane & 15, kk = lane >> 4, k0 = 64 * wv;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      float av[16], bv[16];
#pragma unroll
      for (int s4 = 0; s4 < 16; ++s4) {
        av[s4] = RS[i16 * 516 + k0 + 4 * s4 + kk];
        bv[s4] = P1T[i16 * 516 + k0 + 4 * s4 + kk];
      }
#pragma unroll
      for (int s4 = 0; s4 < 16; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], bv[s4], acc, 0, 0, 0);
      *(floatx4*)(HP + (wv * 64 + lane) * 4) = acc;   // lane-linear: D[4kk + e][i16]
    }
    if (tr && s == n - 1) tr[8 + L + 120] = wall_clock64();
    __syncthreads();
    if (tr && s == n - 1) tr[8 + L + 121] = wall_clock64();
    if (tid < 256) {   // (stream 4·(tid>>6... : element (lane l = tid & 63, e = tid >> 6) of every wave's D
      const int l = tid & 63, e = tid >> 6, sb = 4 * (l >> 4) + e, cc = l & 15;
      float v[8], hsum = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v[g] = HP[(g * 64 + l) * 4 + e];
#pragma unroll
      for (int g = 0; g < 8; ++g) hsum += v[g];
      const float b1c = (m * 16 + cc < Cp && a.post1_b) ? a.post1_b[m * 16 + cc] : 0.f;
      HS[sb * 17 + cc] = (m * 16 + cc < Cp) ? fmaxf(hsum + b1c, 0.f) : 0.f;
    }
    __syncthreads();
    if (tr && s == n - 1) tr[8 + L + 122] = wall_clock64();
    // partial logits over this block's 16 h rows: 16 code columns per MFMA block, blocks wv and
    // wv + 8 of the Q/16: A[i = stream][k = r] = HS, B[k][j = code] = P2S; lane (code, 4 streams)
    {
      const int i16 = lane & 15, kk = lane >> 4;
      float av[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) av[s4] = HS[i16 * 17 + 4 * s4 + kk];
      for (int qb = wv; qb < (Q + 15) / 16; qb += 8) {
        const int q = min(16 * qb + i16, Q - 1);
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], P2S[(4 * s4 + kk) * Q + q], acc, 0, 0, 0);
        if (16 * qb + i16 < Q) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * kk + e < B) put_granule(a.lg + ((long)m * a.B + b0 + 4 * kk + e) * Q + q, tag, acc[e]);
        }
      }
    }
    if (tr && s == n - 1) tr[4] = wall_clock64();
  }
}

__global__ __launch_bounds__(512) void gen_persist_kernel(PersistK a) {
  __shared__ __attribute__((aligned(16))) float sm[G_LDS];
  const int per = a.Bg + P_NH, g = blockIdx.x / per, r = blockIdx.x % per;
  const int b0 = g * a.Bg, Bg = min(a.Bg, a.B - b0);
  long long* stepc = g ? a.gstep + (g - 1) : a.step;
  long long* trace = g ? nullptr : a.trace;
  if (r < Bg) persist_chain(a, sm, b0 + r, stepc, trace);
  else if (r >= a.Bg) persist_head(a, r - a.Bg, sm, b0, Bg, stepc, trace);
  // (a ragged last group leaves chain slots r in [Bg, a.Bg) idle)
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

__global__ void gen_reset_kernel(float* rings, long n_ring, unsigned long long* gran, long n_gran, int* code, int B,
                                 long long* step, int* status) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n_ring; e += (long)gridDim.x * blockDim.x)
    rings[e] = 0.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n_gran; e += (long)gridDim.x * blockDim.x)
    gran[e] = 0ull;   // tags restart at 1 with the step counter
  if (blockIdx.x == 0) {
    for (int b = threadIdx.x; b < B; b += blockDim.x) code[b] = -1;
    if (threadIdx.x == 0) {
      *step = 0;
      *status = 0;
    }
  }
}

}  // namespace

// ---- host side: generation plan ----------------------------------------------------------

#include "../../include/lbwn.h"

struct lbwn_gen_plan {
  lbwn_arch a;
  int B, L, nbl, Cr, Cd, Cs, Cp, Q;
  long long max_steps;
  size_t oRING, oZCAT, oSKP, oHP, oLGP, oLOG, oSTEP, oCODE, oTEACH, oSAMP, oWAV, oGCP, oBSUM, oGIMG, oTRACE, total;
  size_t oGRAN;   // persistent form: granules [zg B·L·32 | sg B·Cs | lg P_NH·B·Q]
  // GEMM form (B > P_MAXB): skip / post1 / post2 as bf16-split MFMA GEMMs over the B streams
  // (split-K partial slabs in oGSPL) instead of the vector GEMVs
  size_t oGSPL = 0;
  int gsplit[3] = {1, 1, 1};
  long n_gran;
  bool trace, persist;
  int pgroups = 1, pbg = 0;   // persistent form: stream groups of pbg <= P_MAXB, each with its own P_NH heads
  long n_gran_core = 0;       // granules before the groups' step counters
  int ksl_skip, ks_skip, ks_h, ks_lg;
  long n_ring;
  long long n_teacher, max_teacher;
  unsigned long long seed;
  int pre_bias;
};

// the per-step GEMM form: large B, shapes the split GEMM takes (N % 4, K % 4, row strides)
static bool gemm_form_ok(const lbwn_gen_plan* p) {
  return !p->persist && p->B > P_MAXB && p->Cs % 4 == 0 && p->Cp % 4 == 0 && p->Q % 4 == 0 && (p->L * p->Cd) % 4 == 0;
}

static size_t gcarve(size_t& cur, size_t bytes) {
  size_t o = cur;
  cur += (bytes + 255) / 256 * 256;
  return o;
}

extern "C" int lbwn_gen_plan_create(const lbwn_arch* a, int B, int64_t max_steps, int64_t max_teacher,
                                    lbwn_gen_plan** out) {
  LBWN_REQUIRE(a && out && B >= 1 && max_steps >= 1 && max_teacher >= 0, "gen_plan_create: bad arguments");
  LBWN_REQUIRE(a->n_res <= 32 && a->n_dil <= 32, "gen: n_res/n_dil must be <= 32");
  LBWN_REQUIRE(a->n_blocks * a->n_block_layers <= G_MAXL, "gen: more than %d layers (tap cache)", G_MAXL);
  LBWN_REQUIRE(a->n_lc_out == 0, "gen: local conditioning is not supported by the cached generator "
                                 "(imodel.py has no LC path)");
  LBWN_REQUIRE(a->n_quant <= 512, "gen: n_quant must be <= 512");
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
  p->oSTEP = gcarve(cur, 16);   // step counter + status word
  p->oCODE = gcarve(cur, 4 * (size_t)B);
  p->oTEACH = gcarve(cur, 4 * (size_t)std::max<int64_t>(1, max_teacher));
  p->oSAMP = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oWAV = gcarve(cur, 4 * (size_t)B * max_steps);
  p->oGCP = gcarve(cur, 4 * (size_t)p->L * B * 64);
  p->oBSUM = gcarve(cur, 4 * (size_t)p->Cs);
  p->oGIMG = gcarve(cur, 4 * (size_t)p->L * GIMG);
  p->oTRACE = gcarve(cur, 8 * (size_t)(2 * p->L + 8 + 128 + 2 * P_NH));
  p->trace = getenv("LBWN_GEN_TRACE") != nullptr;
  // persistent form: every block resident (one 512-thread block per CU), phase A maps
  // (16 skip columns × B streams) onto the threads, the draw's logits fit the tap table's tail
  int dev = 0, ncu = 0;
  const bool have_dev = hipGetDevice(&dev) == hipSuccess &&
                        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
  const char* pe = getenv("LBWN_GEN_PERSIST");
  // B > P_MAXB: ceil(B / P_MAXB) independent groups in the same launch while every block fits
  // (4 x (16 + 32) = 192 blocks for B = 64 on 256 CUs; beyond that the per-step GEMM form)
  p->pgroups = (B + P_MAXB - 1) / P_MAXB;
  p->pbg = (B + p->pgroups - 1) / p->pgroups;
  p->persist = (!pe || strcmp(pe, "0") != 0) && p->L <= P_MAXL && p->Q <= 256 && p->Cs <= 16 * P_NH &&
               p->Cp <= 16 * P_NH && have_dev && p->pgroups * (p->pbg + P_NH) <= ncu;
  p->n_gran_core = (long)B * p->L * 32 + (long)B * p->Cs + (long)P_NH * B * p->Q;
  p->n_gran = p->n_gran_core + p->pgroups;   // + the groups' step counters (zeroed with the granules)
  p->oGRAN = gcarve(cur, 8 * (size_t)p->n_gran);
  if (gemm_form_ok(p)) {
    // split K until ~256 blocks of 128 x 128 tiles (M = B streams is short), >= 4 k-steps of 32 each
    const int Ns[3] = {p->Cs, p->Cp, p->Q}, Ks[3] = {p->L * p->Cd, p->Cs, p->Cp};
    long most = 0;
    for (int i = 0; i < 3; ++i) {
      const int tiles = ((B + 127) / 128) * ((Ns[i] + 127) / 128);
      p->gsplit[i] = std::max(1, std::min(256 / std::max(1, tiles), Ks[i] / 128));
      most = std::max(most, (long)p->gsplit[i] * B * Ns[i]);
    }
    p->oGSPL = gcarve(cur, 4 * (size_t)most);
  }
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
  else if (!strcmp(name, "status")) { *off = p->oSTEP + 8; *bytes = 4; }   // 0, or 5: a persistent hand-off timed out
  else if (!strcmp(name, "trace")) { *off = p->oTRACE; *bytes = 8 * (size_t)(2 * p->L + 8 + 128 + 2 * P_NH); }
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
  gen_reset_kernel<<<256, 256, 0, st>>>(gat<float>(ws, p->oRING), p->n_ring, gat<unsigned long long>(ws, p->oGRAN),
                                        p->n_gran, gat<int>(ws, p->oCODE), p->B, gat<long long>(ws, p->oSTEP),
                                        gat<int>(ws, p->oSTEP + 8));
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

extern "C" int lbwn_gen_is_persistent(const lbwn_gen_plan* p) { return p && p->persist ? 1 : 0; }

static WaveK wave_args(lbwn_gen_plan* p, const lbwn_params* P, void* ws) {
  WaveK c;
  c.pre = P->pre; c.pre_b = P->pre_b; c.img = gat<float>(ws, p->oGIMG);
  c.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
  c.rings = gat<float>(ws, p->oRING); c.zcat = gat<float>(ws, p->oZCAT);
  c.step = gat<long long>(ws, p->oSTEP); c.code = gat<int>(ws, p->oCODE);
  c.trace = nullptr;
  c.B = p->B; c.L = p->L; c.nbl = p->nbl; c.Cr = p->Cr; c.Cd = p->Cd; c.pre_bias = p->pre_bias;
  return c;
}

// Per-step GEMM form (B > P_MAXB): the chain (gen_wave, one workgroup per stream) then the head as
// three bf16-split MFMA GEMMs over all B streams (imodel.py:125-164: skip = Σ_l z_l·SKIP_l + Σb,
// h = relu(relu(skip)·POST1 + b1), logits = h·POST2 + b2) and the sampler.  The K-split vector GEMVs
// re-read every weight per 16-stream group with FMA (B = 256: 211 µs per step).
static int gen_run_gemm(lbwn_gen_plan* p, const lbwn_params* P, void* ws, int n_steps, DrawK d, hipStream_t st) {
  const WaveK c = wave_args(p, P, ws);
  float* S = gat<float>(ws, p->oSKP);     // [B][Cs]   (the GEMV partial buffers are larger)
  float* H = gat<float>(ws, p->oHP);      // [B][Cp]
  float* LG = gat<float>(ws, p->oLGP);    // [B][Q] logits with b2
  float* SPL = gat<float>(ws, p->oGSPL);
  lbwn_gemm_args sk, p1, p2;
  memset(&sk, 0, sizeof(sk));
  sk.A = c.zcat; sk.lda = (long)p->L * p->Cd; sk.B = P->skip; sk.ldb = p->Cs; sk.C = S; sk.ldc = p->Cs;
  sk.M = p->B; sk.N = p->Cs; sk.K = p->L * p->Cd; sk.bias = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr;
  sk.step_advance = gat<long long>(ws, p->oSTEP);   // the sampler reads step - 1
  p1 = sk;
  p1.step_advance = nullptr;
  p1.A = S; p1.lda = p->Cs; p1.relu_a = 1; p1.B = P->post1; p1.ldb = p->Cp; p1.C = H; p1.ldc = p->Cp;
  p1.N = p->Cp; p1.K = p->Cs; p1.bias = P->post1_b; p1.relu_out = 1;
  p2 = p1;
  p2.A = H; p2.lda = p->Cp; p2.relu_a = 0; p2.B = P->post2; p2.ldb = p->Q; p2.C = LG; p2.ldc = p->Q;
  p2.N = p->Q; p2.K = p->Cp; p2.bias = P->post2_b; p2.relu_out = 0;
  d.part = LG; d.parts = 1; d.bias = nullptr;   // b2 added by the GEMM
  for (int i = 0; i < n_steps; ++i) {
    gen_wave_kernel<<<p->B, 512, 0, st>>>(c);
    LBWN_CHECK_LAUNCH();
    if (int e = lbwn_gemm_launch(sk, 1, 0, p->gsplit[0], SPL, st)) return e;
    if (int e = lbwn_gemm_launch(p1, 1, 0, p->gsplit[1], SPL, st)) return e;
    if (int e = lbwn_gemm_launch(p2, 1, 0, p->gsplit[2], SPL, st)) return e;
    gen_sample_kernel<<<p->B, 64, 0, st>>>(d, c.step);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lbwn_gen_run(lbwn_gen_plan* p, const lbwn_params* P, void* ws, int n_steps, void* stream) {
  LBWN_REQUIRE(p && P && ws && n_steps >= 0, "gen_run: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  DrawK d;
  memset(&d, 0, sizeof(d));
  d.Q = p->Q; d.B = p->B; d.bias = P->post2_b;
  d.logits = gat<float>(ws, p->oLOG); d.samples = gat<int>(ws, p->oSAMP); d.wav = gat<float>(ws, p->oWAV);
  d.max_steps = p->max_steps; d.teacher = gat<int>(ws, p->oTEACH); d.n_teacher = p->n_teacher; d.seed = p->seed;
  d.code = gat<int>(ws, p->oCODE);
  if (p->persist) {
    if (n_steps == 0) return 0;
    PersistK k;
    memset(&k, 0, sizeof(k));
    k.pre = P->pre; k.pre_b = P->pre_b; k.img = gat<float>(ws, p->oGIMG);
    k.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
    k.rings = gat<float>(ws, p->oRING); k.step = gat<long long>(ws, p->oSTEP); k.code_in = gat<int>(ws, p->oCODE);
    k.B = p->B; k.L = p->L; k.nbl = p->nbl; k.Cr = p->Cr; k.Cd = p->Cd; k.pre_bias = p->pre_bias; k.n_steps = n_steps;
    unsigned long long* g = gat<unsigned long long>(ws, p->oGRAN);
    k.zg = g; k.sg = g + (long)p->B * p->L * 32; k.lg = k.sg + (long)p->B * p->Cs;
    k.Cs = p->Cs; k.Cp = p->Cp; k.Q = p->Q;
    k.skipw = P->skip; k.bsum = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr;
    k.post1 = P->post1; k.post1_b = P->post1_b; k.post2 = P->post2;
    k.draw = d;
    k.status = gat<int>(ws, p->oSTEP + 8);
    k.trace = p->trace ? gat<long long>(ws, p->oTRACE) : nullptr;
    k.Bg = p->pbg;
    k.gstep = reinterpret_cast<long long*>(g + p->n_gran_core);
    gen_persist_kernel<<<p->pgroups * (p->pbg + P_NH), 512, 0, st>>>(k);
    LBWN_CHECK_LAUNCH();
    gen_decode_kernel<<<std::max(1, std::min(1024, (int)(((long long)p->B * n_steps + 255) / 256))), 256, 0, st>>>(
        d.samples, d.wav, k.step, p->B, p->max_steps, n_steps, p->Q);
    LBWN_CHECK_LAUNCH();
    return 0;
  }
  if (p->oGSPL && !p->trace && lbwn_gemm_mode() == 1) return gen_run_gemm(p, P, ws, n_steps, d, st);
  WaveK c;
  c.pre = P->pre; c.pre_b = P->pre_b; c.img = gat<float>(ws, p->oGIMG);
  c.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
  c.rings = gat<float>(ws, p->oRING); c.zcat = gat<float>(ws, p->oZCAT);
  c.step = gat<long long>(ws, p->oSTEP); c.code = gat<int>(ws, p->oCODE);
  c.trace = p->trace ? gat<long long>(ws, p->oTRACE) : nullptr;
  c.B = p->B; c.L = p->L; c.nbl = p->nbl; c.Cr = p->Cr; c.Cd = p->Cd; c.pre_bias = p->pre_bias;
  // skip = z_cat·SKIPcat (+Σb and relu applied by the consumer), h = relu(relu(skip)·POST1 + b1),
  // logits = h·POST2 + b2 (summed in the sampler)
  GemvK sk = {}, p1 = {}, p2 = {};
  memset(&sk, 0, sizeof(sk));
  sk.in = c.zcat; sk.ldin = (long)p->L * p->Cd; sk.W = P->skip; sk.ldw = p->Cs; sk.out_part = gat<float>(ws, p->oSKP);
  sk.B = p->B; sk.K = p->L * p->Cd; sk.N = p->Cs; sk.KSL = p->ksl_skip;
  sk.step_advance = gat<long long>(ws, p->oSTEP);   // the sampler reads step - 1
  p1 = sk;
  p1.step_advance = nullptr;
  p1.in = nullptr; p1.in_part = sk.out_part; p1.in_parts = p->ks_skip; p1.in_bias = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr;
  p1.relu_in = 1; p1.W = P->post1; p1.ldw = p->Cp; p1.out_part = gat<float>(ws, p->oHP); p1.K = p->Cs; p1.N = p->Cp; p1.KSL = 32;
  p2 = p1;
  p2.in_part = p1.out_part; p2.in_parts = p->ks_h; p2.in_bias = P->post1_b; p2.relu_in = 1;
  p2.W = P->post2; p2.ldw = p->Q; p2.out_part = gat<float>(ws, p->oLGP); p2.K = p->Cp; p2.N = p->Q; p2.KSL = 32;
  d.part = p2.out_part; d.parts = p->ks_lg;
  const dim3 gsk((sk.N + 63) / 64, p->ks_skip), gp1((p1.N + 63) / 64, (p1.K + 31) / 32), gp2((p2.N + 63) / 64, (p2.K + 31) / 32);
  if (p->trace) {   // GEMV stamps after the wave kernel's: [skip | post1 | post2] × 8
    long long* tb = gat<long long>(ws, p->oTRACE) + 2 * p->L + 8;
    sk.trace = tb; p1.trace = tb + 8; p2.trace = tb + 16;
  }
  for (int i = 0; i < n_steps; ++i) {
    gen_wave_kernel<<<p->B, 512, 0, st>>>(c);
    gen_gemv_kernel<<<gsk, 256, 0, st>>>(sk);
    gen_gemv_kernel<<<gp1, 256, 0, st>>>(p1);
    gen_gemv_kernel<<<gp2, 256, 0, st>>>(p2);
    gen_sample_kernel<<<p->B, 64, 0, st>>>(d, c.step);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}

