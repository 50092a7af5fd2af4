// Cached single-step autoregressive generation (imodel.py:61-272).
//
// Per generated sample, all state stays on device so a chunk of steps can be captured in a
// hipGraph and replayed: the step counter, the per-layer lookback rings (the generation
// form of the D-separation cache: layer l keeps its last d inputs, slot t mod d, replacing
// imodel's shift-by-chunk buffers imodel.py:88-98, :190-207), the next input code, the
// teacher vector and a counter-based RNG.  One step = three launches:
//   gen_wave     one workgroup per stream: four compute waves draw the PREVIOUS step (Σ post2
//                partials + b2, inverse-CDF with u = hash(seed, stream, step), µ-law decode, next
//                input = teacher[t] or the draw: imodel.py:167-187, :260-269), then run PRE row
//                (+bias), 50 × [dilated conv, gate, residual] while four loader waves stream the
//                per-layer weight images into an LDS ring by LDS-DMA, several layers ahead.  Each
//                z_l leaves as tagged 8-byte granules; skip helper blocks of the same launch
//                (layer pairs of SKIPcat) poll them and accumulate the skip sum as the chain runs
//   gen_gemv × 2 K-split row-vector products with deterministic partial sums:
//                h = relu(relu(Σ skip partials + Σb)·POST1 + b1), logits partials = h·POST2
// (the last step of a run is drawn by gen_sample, one wave per stream, same draw code)
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
//     conv      lane = (c, sg = sig|gate, kq = k-quarter): 16 FMAs over its quarter of
//               [x[t-d] | x[t]] (4 weight + 4 broadcast input ds_read_b128), the quarters summed
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
constexpr int GI_W = 16 * 256;              // conv: [w 4][m 4][lane 64][4]  W[16kq+4m+j][32sg+8w+c]
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

// ---- the draw (imodel.py:167-187, :260-269) ----------------------------------------------
// logits[c] = Σ_p part[p][b][c] + bias[c] (fixed order), then the first k with
// cumsum(e)[k] > u·Σe, e = exp(logits - max), u = hash(seed, stream, step).  Wave-level only
// (lane = a contiguous run of ceil(Q/64) codes, shuffles, no workgroup barrier), so the four
// compute waves of a gen_wave block all draw the same code without exchanging it, and the
// standalone gen_sample_kernel (one wave per stream) runs the identical instruction sequence
// (oracle/wavenet_ref.py sample_from_logits restates the transform).
struct DrawK {
  const float* part; int parts; const float* bias;   // partials [parts][B][Q]
  int Q, B;
  float* logits; int* samples; float* wav; long long max_steps;
  const int* teacher; long long n_teacher; unsigned long long seed; int* code;
};

LBWN_DEV uint64_t splitmix(uint64_t seed, uint64_t stream, uint64_t step) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ULL + (stream << 32) + step + 0x632BE59BD9B4E019ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// returns the next input code of stream b after step t (the teacher's or the draw); the
// writing wave stores logits, the sample, its µ-law decode and code[b]
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
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    const bool ok = j < per && c0 + j < Q;
    if (a.bias) v[j] += bv[j];
    if (ok) mx = fmaxf(mx, v[j]);
    if (ok && write) a.logits[(long)b * Q + c0 + j] = v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float e[MP], loc = 0.f;
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    e[j] = (j < per && c0 + j < Q) ? expf(v[j] - mx) : 0.f;
    loc += e[j];
  }
  float incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float s = __shfl_up(incl, o);
    if (lane >= o) incl += s;
  }
  const float total = __shfl(incl, 63);
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
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) found = min(found, __shfl_xor(found, o));
  if (found >= Q) found = Q - 1;
  const int next = (t < a.n_teacher) ? a.teacher[t] : found;   // imodel.py:260-269
  if (write && lane == 0) {
    if (t < a.max_steps) {
      a.samples[(long)b * a.max_steps + t] = found;
      const float mu = (float)(Q - 1), inv = 1.f / mu;               // ops.py:12-20
      const float aa = (2.f * (float)found - 1.f) * inv - 1.f;
      const float sg = aa > 0.f ? 1.f : (aa < 0.f ? -1.f : 0.f);
      a.wav[(long)b * a.max_steps + t] = sg * (powf(1.f + mu, fabsf(aa)) - 1.f) * inv;
    }
    a.code[b] = next;
  }
  return next;
}

struct WaveK {
  const float* pre; const float* pre_b; const float* img; const float* gc_proj;
  float* rings; const long long* step; const int* code;
  int B, L, nbl, Cr, Cd, pre_bias;
  // z_l of every stream as {z, tag = step+1} granules [B][L][32] (one 8-B sc1 store each), read
  // by the skip helper blocks of the same launch (blockIdx >= B): helper j owns layers
  // [LG·j, LG·j+LG) of SKIPcat [L·Cd][Cs] and writes its partial skip sum [j][B][Cs]
  unsigned long long* zg; const float* skipw; float* skip_part; int Cs, LG;
  int* status;
  // fused draw: this launch first draws step t-1 of its stream (the previous step's post2
  // partials), so the sampler launch and its boundary leave the per-step chain
  int fuse_draw; DrawK draw;
  long long* trace;   // non-null (LBWN_GEN_TRACE set at plan creation): stream 0's cycle stamps
};

constexpr long long G_SPIN_TIMEOUT = 400000000LL;   // wall_clock64 ticks (100 MHz) = 4 s

// skip helper j: per group of 16 streams and per owned layer, poll the 16×Cd z granules (one
// per thread), stage them in LDS, and accumulate Σ_k z[b][k]·SKIP[l·Cd+k][n] for column n =
// threadIdx.x; the layer's weight column is loaded before the poll so its latency hides there
LBWN_DEV void skip_helper(const WaveK& a, int j, long long t, float* sm) {
  const int tid = threadIdx.x, L = a.L, Cd = a.Cd, Cs = a.Cs, B = a.B;
  const int l0 = j * a.LG, l1 = min(L, l0 + a.LG);
  const unsigned tag = (unsigned)(t + 1);
  const int n = min(tid, Cs - 1), gb = tid >> 5, gk = tid & 31;
  for (int g0 = 0; g0 < B; g0 += 16) {
    const int nb = min(16, B - g0);
    float acc[16];
#pragma unroll
    for (int bb = 0; bb < 16; ++bb) acc[bb] = 0.f;
    int buf = 0;
    for (int l = l0; l < l1; ++l, buf ^= 1) {
      float w[32];
      const float* S = a.skipw + (long)l * Cd * Cs + n;
#pragma unroll
      for (int k = 0; k < 32; ++k) w[k] = S[(long)min(k, Cd - 1) * Cs];
#pragma unroll
      for (int k = 0; k < 32; ++k)
        if (k >= Cd) w[k] = 0.f;
      float zv = 0.f;
      if (gb < nb && gk < Cd) {
        const unsigned long long* gp = a.zg + ((long)(g0 + gb) * L + l) * 32 + gk;
        long long ts = 0;
        for (;;) {
          const unsigned long long g = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(g >> 32) == tag) { zv = __uint_as_float((unsigned)g); break; }
          const long long now = wall_clock64();
          if (ts == 0) ts = now;
          else if (now - ts > G_SPIN_TIMEOUT) {
            __hip_atomic_store(a.status, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      const bool trh = a.trace && tid == 0 && blockIdx.x == gridDim.x - 1 && l - l0 < 2 && g0 == 0;
      if (trh) a.trace[2 * L + 12 + 2 * (l - l0)] = wall_clock64();
      float* ZS = sm + buf * 512;   // [16 streams][32]; double-buffered: one barrier per layer
      ZS[tid] = zv;
      __syncthreads();
#pragma unroll
      for (int bb = 0; bb < 16; ++bb) {
        if (bb < nb) {
          const floatx4* zr = (const floatx4*)(ZS + bb * 32);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const floatx4 z4 = zr[q];
            acc[bb] = fmaf(z4[0], w[4 * q], acc[bb]);
            acc[bb] = fmaf(z4[1], w[4 * q + 1], acc[bb]);
            acc[bb] = fmaf(z4[2], w[4 * q + 2], acc[bb]);
            acc[bb] = fmaf(z4[3], w[4 * q + 3], acc[bb]);
          }
        }
      }
    }
    if (a.trace && tid == 0 && blockIdx.x == gridDim.x - 1 && g0 == 0) a.trace[2 * L + 13] = wall_clock64();
    if (tid < Cs) {
#pragma unroll
      for (int bb = 0; bb < 16; ++bb)
        if (bb < nb) a.skip_part[((long)j * B + g0 + bb) * Cs + tid] = acc[bb];
    }
  }
}

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

  if (b >= a.B) {   // ---- skip helper blocks
    const bool trh = a.trace && threadIdx.x == 0 && b == gridDim.x - 1;
    if (trh) a.trace[2 * L + 10] = wall_clock64();
    skip_helper(a, b - a.B, t, sm);
    if (trh) a.trace[2 * L + 11] = wall_clock64();
    return;
  }

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
  if (tr) { a.trace[0] = clock64(); a.trace[2 * L + 8] = wall_clock64(); }
  long long* trs = (a.trace && w == 0 && lane == 0) ? a.trace + 2 * L + 40 + 3 * b : nullptr;
  if (trs) trs[0] = wall_clock64();
  // step input: PRE row of the previous draw (+ PRE_BIAS); the zero vector at step 0.  With
  // fuse_draw every compute wave draws step t-1 itself (wave 0 writes), while the loader waves'
  // first taps and weight slots are in flight
  int code;
  if (a.fuse_draw)
    code = a.draw.Q > 256 ? draw_wave<8>(a.draw, b, t - 1, w == 0) : draw_wave<4>(a.draw, b, t - 1, w == 0);
  else
    code = a.code[b];
  float x = 0.f;    // x[rc] of the current layer input
  if (rc < Cr) {
    if (code >= 0) x = a.pre[(long)code * Cr + rc];
    if (a.pre_bias && a.pre_b) x += a.pre_b[rc];
  }
  if (lane < 32) XW[rc] = x;
  if (tr) a.trace[1] = clock64();
  if (trs) trs[1] = wall_clock64();
  const int xin_off = kq < 2 ? 16 * kq : 16 * (kq - 2);
  long roff = 0;   // ring offset of layer l
  int bl = 0;      // l % nbl
  lds_barrier();   // barrier -1: taps and slot 0 landed, every wave's XW written
  if (tr) a.trace[2] = clock64();
  for (int l = 0; l < L; ++l) {
    const float* S = RING + (l % G_NS) * G_SLOT;
    const float* xin = (kq < 2 ? XP + l * 32 : XW) + xin_off;
    floatx4 wv[4], xv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      wv[m] = *(const floatx4*)(S + (w * 4 + m) * 256 + lane * 4);
      xv[m] = *(const floatx4*)(xin + 4 * m);
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
    const float z = tanhf_(sg ? vp : v) * sigmoidf_(sg ? v : vp);
    float* Zl = Z + (l & 1) * 32;
    if (lead) {
      Zl[ch] = z;
      if (ch < Cd)   // granule for the skip helpers: fire-and-forget, no wait on the chain
        __hip_atomic_store(a.zg + ((long)b * L + l) * 32 + ch,
                           ((unsigned long long)(unsigned)(t + 1) << 32) | __float_as_uint(z), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
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
  if (tr) a.trace[2 * L + 9] = wall_clock64();
  if (trs) trs[2] = wall_clock64();
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
      const int k = 16 * kq + 4 * m + j, tap = k >> 5, in = k & 31, oc = 8 * w + c;
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

// the step's draw when it is not fused into the next gen_wave launch (the last step of a run):
// one wave per stream, t = *step - 1 (post1 advanced the counter)
__global__ __launch_bounds__(64) void gen_sample_kernel(DrawK a, const long long* step) {
  const long long t = *step - 1;
  if (a.Q > 256) draw_wave<8>(a, blockIdx.x, t, true);
  else draw_wave<4>(a, blockIdx.x, t, true);
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

__global__ void gen_reset_kernel(float* rings, long n_ring, int* code, int B, long long* step, int* status) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n_ring; e += (long)gridDim.x * blockDim.x)
    rings[e] = 0.f;
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
  size_t oRING, oZG, oSKP, oHP, oLGP, oLOG, oSTEP, oCODE, oTEACH, oSAMP, oWAV, oGCP, oBSUM, oGIMG, oTRACE, total;
  bool trace;
  int lg_skip, ks_skip, ks_h, ks_lg;
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
  LBWN_REQUIRE(a->n_skip <= 512, "gen: n_skip must be <= 512 (one skip column per helper thread)");
  LBWN_REQUIRE(a->n_quant <= 512, "gen: n_quant must be <= 512");
  LBWN_REQUIRE(a->n_blocks * a->n_block_layers <= G_MAXL, "gen: more than %d layers (tap cache)", G_MAXL);
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
  p->oZG = gcarve(cur, 8 * (size_t)B * p->L * 32);   // z granules {z, step+1}
  // K-split GEMV partials: skip (K = L·Cd, 64-row slices), post1 and post2 (32-row slices)
  p->lg_skip = 2;                                    // layers per skip helper block
  p->ks_skip = (p->L + p->lg_skip - 1) / p->lg_skip;
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
  p->oTRACE = gcarve(cur, 8 * (size_t)(2 * p->L + 40 + 3 * p->B));
  p->trace = getenv("LBWN_GEN_TRACE") != nullptr;
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
  else if (!strcmp(name, "status")) { *off = p->oSTEP + 8; *bytes = 4; }   // 0, or 5: a skip helper's granule poll timed out
  else if (!strcmp(name, "trace")) { *off = p->oTRACE; *bytes = 8 * (size_t)(2 * p->L + 40 + 3 * p->B); }
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
                                        gat<long long>(ws, p->oSTEP), gat<int>(ws, p->oSTEP + 8));
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
  memset(&c, 0, sizeof(c));
  c.pre = P->pre; c.pre_b = P->pre_b; c.img = gat<float>(ws, p->oGIMG);
  c.gc_proj = p->a.n_gc_embed > 0 ? gat<float>(ws, p->oGCP) : nullptr;
  c.rings = gat<float>(ws, p->oRING);
  c.step = gat<long long>(ws, p->oSTEP); c.code = gat<int>(ws, p->oCODE);
  c.trace = p->trace ? gat<long long>(ws, p->oTRACE) : nullptr;
  c.B = p->B; c.L = p->L; c.nbl = p->nbl; c.Cr = p->Cr; c.Cd = p->Cd; c.pre_bias = p->pre_bias;
  c.zg = gat<unsigned long long>(ws, p->oZG); c.skipw = P->skip; c.skip_part = gat<float>(ws, p->oSKP);
  c.Cs = p->Cs; c.LG = p->lg_skip; c.status = gat<int>(ws, p->oSTEP + 8);
  // skip = Σ helper partials (+Σb, relu: post1's input), h = relu(relu(skip)·POST1 + b1),
  // logits = h·POST2 + b2 (summed by the draw); post1 advances the step counter
  GemvK p1, p2;
  memset(&p1, 0, sizeof(p1));
  p1.in_part = c.skip_part; p1.in_parts = p->ks_skip; p1.in_bias = P->skip_b ? gat<float>(ws, p->oBSUM) : nullptr;
  p1.relu_in = 1; p1.W = P->post1; p1.ldw = p->Cp; p1.out_part = gat<float>(ws, p->oHP);
  p1.B = p->B; p1.K = p->Cs; p1.N = p->Cp; p1.KSL = 32;
  p1.step_advance = gat<long long>(ws, p->oSTEP);
  p2 = p1;
  p2.step_advance = nullptr;
  p2.in_part = p1.out_part; p2.in_parts = p->ks_h; p2.in_bias = P->post1_b; p2.relu_in = 1;
  p2.W = P->post2; p2.ldw = p->Q; p2.out_part = gat<float>(ws, p->oLGP); p2.K = p->Cp; p2.N = p->Q; p2.KSL = 32;
  DrawK& d = c.draw;
  d.part = p2.out_part; d.parts = p->ks_lg; d.bias = P->post2_b; d.Q = p->Q; d.B = p->B;
  d.logits = gat<float>(ws, p->oLOG); d.samples = gat<int>(ws, p->oSAMP); d.wav = gat<float>(ws, p->oWAV);
  d.max_steps = p->max_steps; d.teacher = gat<int>(ws, p->oTEACH); d.n_teacher = p->n_teacher; d.seed = p->seed;
  d.code = gat<int>(ws, p->oCODE);
  const dim3 gp1((p1.N + 63) / 64, (p1.K + 31) / 32), gp2((p2.N + 63) / 64, (p2.K + 31) / 32);
  if (p->trace) {   // GEMV stamps after the wave kernel's: [unused | post1 | post2] × 8
    long long* tb = gat<long long>(ws, p->oTRACE) + 2 * p->L + 8;
    p1.trace = tb + 8; p2.trace = tb + 16;
  }
  // per step: gen_wave (chains + skip helpers; from the second step of the run on, it first
  // draws the previous step), post1, post2; the run's last step is drawn by gen_sample
  for (int i = 0; i < n_steps; ++i) {
    c.fuse_draw = i > 0;
    gen_wave_kernel<<<p->B + p->ks_skip, 512, 0, st>>>(c);
    gen_gemv_kernel<<<gp1, 256, 0, st>>>(p1);
    gen_gemv_kernel<<<gp2, 256, 0, st>>>(p2);
    LBWN_CHECK_LAUNCH();
  }
  if (n_steps > 0) {
    gen_sample_kernel<<<p->B, 64, 0, st>>>(c.draw, c.step);
    LBWN_CHECK_LAUNCH();
  }
  return 0;
}
