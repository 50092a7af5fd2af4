// One WaveNet residual layer, forward and backward (tmodel.py:117-184, :313-325).
//
// Layout: activations are channels-last rows; x_l lives in a per-stream buffer
// [B][H+T][Cr] whose first H rows are a halo: rows [H-d, H) hold SAVE_l, so the dilated
// tap x[t-d] (or SAVE for t<d, tmodel.py:122-127) is simply row H+t-d.  A block owns 128
// consecutive positions of one stream (grid-stride over such tiles); both taps are staged
// into LDS with coalesced 16-B loads (Xp = rows t-d, Xc = rows t), then each wave computes
// a 32-position tile with v_mfma_f32_32x32x2_f32 in the TRANSPOSED orientation (channels on
// MFMA rows, positions on lanes) so that the gate output z is already the B operand of the
// residual / dx products (no lane shuffles):
//   vᵀ[64 × 32pos] = Wcatᵀ[64 out × 64 in] · [x[t-d] | x[t]]ᵀ   (sig rows 0-31, gate 32-63)
//   zᵀ = tanh(v_sig)·σ(v_gate);  x_{l+1}ᵀ = x_lᵀ + RESᵀ·zᵀ + b_res
// Weights arrive pre-packed per layer in the exact padded LDS image (lbwn_pack_layers), so
// staging is a straight 16-B copy.  Channel counts up to 32 are supported (zero-padded).
#include <string.h>

#include "common.h"
#include "kernels.h"
#include "prologue.h"

namespace {

constexpr int LP = LBWN_LAYER_POS;  // positions per tile (4 waves × 32)
constexpr int XS = 36;              // padded LDS row for 32-channel tiles (b128 conflict-free)
constexpr int WS = 68;              // padded row of the [64 in][64 out] conv weight image
constexpr int DS = 68;              // dv tile row [pos][64]
constexpr int WIMG = 64 * WS + 32 * XS + 96;  // packed per-layer image (floats), multiple of 4
constexpr int SLAB = 2048 + 2048 + 1024 + 96;
constexpr int RED_PARTS = 32;       // deferred reduction: parts prefetched per thread (8 lanes × 32)
// Timing-only ablation switches (variant builds: make EXTRA=-DLBWN_ABL=<bits> OBJDIR=... OUT=...);
// 0 in every real build.
#ifndef LBWN_ABL
#define LBWN_ABL 0
#endif
// LDS bank-conflict attribution (round 3, counter-only variant builds with EXTRA=-DLBWN_CONF=<bits>,
// profiles/r03_lds_conf_*.txt): bit b sends one group of
// chain_bwd_x3_kernel's LDS accesses to a conflict-free address (reads: a wave-uniform broadcast,
// writes (2048): lane-contiguous 16-B slots); the outputs are wrong, SQ_LDS_BANK_CONFLICT's drop
// per bit is that group's share.  0 in every real build.
#ifndef LBWN_CONF
#define LBWN_CONF 0
#endif
#define CONF(bit) ((LBWN_CONF & (bit)) != 0)

// Compact kernel arguments (the full lbwn_layer_args by value spilled ~100 SGPRs).
struct FwdK {
  const float* x_in; float* x_out; float* z; const float* wpack;
  const float* gc_tab; const int* ids; const float* cond;
  long ldz, ldcond, gc_ld;
  int B, T, H, d, Cr, Cd;
};
struct BwdK {
  const float* x_in; const float* wpack; const float* dz_skip;
  const float* g_a; const float* g_c0; float* out_a; float* out_c0; float* slab;
  const float* gc_tab; const int* ids; const float* cond; float* dv_out; float* gc_dtab;
  long lddz, ldcond, lddv, gc_ld;
  int B, T, H, d, Cr, Cd, g_d, slab_stride;
};
// Standalone slab reduction (runs on an auxiliary stream, off the layer chain).
struct RedK {
  const float* slab; float* dsig; float* dgate; float* dres; float* dbsig; float* dbgate; float* dbres;
  int nparts, stride, Cr, Cd;
};

// ---- weight packing ---------------------------------------------------------------------
// image: Ws[k = tap*32 + in][out (sig 0..31 | gate 32..63)] (row WS), Rs[c][o] (row XS),
//        bs[64] (sig | gate), br[32]

__global__ void pack_layers_kernel(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                   const float* res, const float* res_b, float* out, int Cr, int Cd) {
  const int l = blockIdx.x;
  const float* ws = sig + (long)l * 2 * Cr * Cd;
  const float* wg = gate + (long)l * 2 * Cr * Cd;
  const float* wr = res + (long)l * Cd * Cr;
  float* img = out + (long)l * WIMG;
  for (int e = threadIdx.x; e < 64 * WS; e += blockDim.x) {
    const int k = e / WS, o = e % WS;
    const int tap = k >> 5, in = k & 31, oc = o & 31;
    float v = 0.f;
    if (o < 64 && in < Cr && oc < Cd) v = (o < 32 ? ws : wg)[(tap * Cr + in) * Cd + oc];
    img[e] = v;
  }
  for (int e = threadIdx.x; e < 32 * XS; e += blockDim.x) {
    const int c = e / XS, o = e % XS;
    img[64 * WS + e] = (c < Cd && o < Cr) ? wr[c * Cr + o] : 0.f;
  }
  if (threadIdx.x < 96) {
    const int i = threadIdx.x;
    float v = 0.f;
    if (i < 64) {
      const float* bb = i < 32 ? sig_b : gate_b;
      if (bb && (i & 31) < Cd) v = bb[(long)l * Cd + (i & 31)];
    } else if (res_b && i - 64 < Cr) {
      v = res_b[(long)l * Cr + (i - 64)];
    }
    img[64 * WS + 32 * XS + i] = v;
  }
}

// Split image for the forward chain's bf16-split conv / residual, bf16 units:
//   WT[o (sig 0..31 | gate 32..63)][tap][plane][in 0..31]  (row XW_ROW = 192 + 8 pad: rows 100
//     dwords apart, conflict-free b128 fragment reads)
//   RT[out][plane][kk]  (row XR_ROW = 96 + 8 pad), kk = 16s + 8h + j holds z channel
//     16s + 8(j>>2) + 4h + (j&3): the k order of a 32x32 accumulator used as the B operand
//     (registers 8s..8s+7 of lane half h), cdna_hip_programming §3
//   then bs[64], br[32] as f32.
constexpr int XW_ROW = 200, XR_ROW = 104;
constexpr int XB_OFF = 64 * XW_ROW + 32 * XR_ROW;             // bf16 offset of the f32 biases
// bf16 elements per layer image, padded to 32 whole 1-KiB LDS-DMA pieces (the pad is never read)
constexpr int XIMG_US = (XB_OFF + 2 * 96 + 511) / 512 * 512;
constexpr int XIMG_F = XIMG_US / 2;                            // = 8192 floats
static_assert(XIMG_F % 256 == 0 && XB_OFF % 8 == 0, "x3 image alignment");

// Split image of a layer's LC projection for the forward chain's in-chain LC term
// (tmodel.py:155-160: v_k += lc·LC_k), bf16 units: LCT[o (sig 0..31 | gate 32..63)][plane][k 0..79]
// in rows of LC_ROW = 3·80 + 8 pad (124 dwords: 4·odd, so every 16-lane ds_read_b128 group of the
// A-fragment reads is conflict-free, MI355X_MICROARCH §LDS), k >= n_lc_out zero.  31 KiB per layer:
// exactly 31 LDS-DMA pieces.  Used when 64 < n_lc_out <= 80 (LC_K = 5 k-steps of 16).
constexpr int LC_K = 5, LC_KP = 16 * LC_K, LC_ROW = 3 * LC_KP + 8;
constexpr int LCIMG_US = 64 * LC_ROW;                          // bf16 elements per layer image
constexpr int LCIMG_F = LCIMG_US / 2;                          // = 7936 floats
static_assert(LCIMG_F % 256 == 0, "LC image: whole 1-KiB DMA pieces");

LBWN_DEV void pack_lc_x3_body(int l, const float* lsig, const float* lgate, unsigned short* out, int Lo, int Cd) {
  unsigned short* img = out + (long)l * LCIMG_US;
  for (int e = threadIdx.x; e < 64 * (LC_ROW / 2); e += blockDim.x) {
    const int o = e / (LC_ROW / 2), kk = 2 * (e % (LC_ROW / 2));
    unsigned short* row = img + o * LC_ROW;
    if (kk >= LC_KP) {   // pad columns (never read) and the plane slots past k: written as part of planes below
      if (kk >= 3 * LC_KP) *(unsigned*)(row + kk) = 0u;
      continue;
    }
    const float* w = (o < 32 ? lsig : lgate) + (long)l * Lo * Cd;
    const int oc = o & 31;
    floatx2 x = {0.f, 0.f};
    if (oc < Cd) {
      if (kk < Lo) x[0] = w[(long)kk * Cd + oc];
      if (kk + 1 < Lo) x[1] = w[(long)(kk + 1) * Cd + oc];
    }
    unsigned hi, mi, lo;
    split2(x, hi, mi, lo);
    *(unsigned*)(row + kk) = hi;
    *(unsigned*)(row + LC_KP + kk) = mi;
    *(unsigned*)(row + 2 * LC_KP + kk) = lo;
  }
}

LBWN_DEV void pack_x3_body(int l, const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                          const float* res, const float* res_b, unsigned short* out, int Cr, int Cd) {
  const float* ws = sig + (long)l * 2 * Cr * Cd;
  const float* wg = gate + (long)l * 2 * Cr * Cd;
  const float* wr = res + (long)l * Cd * Cr;
  unsigned short* img = out + (long)l * XIMG_US;
  // WT: pairs of consecutive input channels
  for (int e = threadIdx.x; e < 64 * 2 * 16; e += blockDim.x) {
    const int o = e >> 5, tap = (e >> 4) & 1, in = 2 * (e & 15), oc = o & 31;
    const float* w = o < 32 ? ws : wg;
    floatx2 x = {0.f, 0.f};
    if (oc < Cd) {
      if (in < Cr) x[0] = w[(tap * Cr + in) * Cd + oc];
      if (in + 1 < Cr) x[1] = w[(tap * Cr + in + 1) * Cd + oc];
    }
    unsigned h, m, lo;
    split2(x, h, m, lo);
    unsigned short* row = img + o * XW_ROW + tap * 96 + in;
    *(unsigned*)(row) = h;
    *(unsigned*)(row + 32) = m;
    *(unsigned*)(row + 64) = lo;
  }
  // RT: kk pairs (kk, kk+1) hold z channels c, c+1 (same j>>2 group)
  for (int e = threadIdx.x; e < 32 * 16; e += blockDim.x) {
    const int o = e >> 4, kk = 2 * (e & 15);
    const int s2 = kk >> 4, hh = (kk >> 3) & 1, j = kk & 7;
    const int c = 16 * s2 + 8 * (j >> 2) + 4 * hh + (j & 3);
    floatx2 x = {0.f, 0.f};
    if (o < Cr) {
      if (c < Cd) x[0] = wr[c * Cr + o];
      if (c + 1 < Cd) x[1] = wr[(c + 1) * Cr + o];
    }
    unsigned h, m, lo;
    split2(x, h, m, lo);
    unsigned short* row = img + 64 * XW_ROW + o * XR_ROW + kk;
    *(unsigned*)(row) = h;
    *(unsigned*)(row + 32) = m;
    *(unsigned*)(row + 64) = lo;
  }
  if (threadIdx.x < 96) {
    const int i = threadIdx.x;
    float v = 0.f;
    if (i < 64) {
      const float* bb = i < 32 ? sig_b : gate_b;
      if (bb && (i & 31) < Cd) v = bb[(long)l * Cd + (i & 31)];
    } else if (res_b && i - 64 < Cr) {
      v = res_b[(long)l * Cr + (i - 64)];
    }
    ((float*)(img + XB_OFF))[i] = v;
  }
}

// ---- LDS staging ---------------------------------------------------------------------

// dst[r][0..31] = x row (t0 + r + shift) of the halo buffer xb, zero if t0+r >= T.
// orders this wave's LDS writes before its later LDS reads of another lane's data (LDS ops of
// one wave are performed in issue order; this stops hipcc from reordering them) — no barrier
LBWN_DEV void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

LBWN_DEV void stage_rows(float* dst, const float* __restrict__ xb, int t0, int shift, int T, int H, int C,
                         int tid) {
  if (C == 32) {
    floatx4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      const int r = e >> 3, c4 = (e & 7) * 4;
      // unconditional load of a clamped row, then select: a predicated load would sit behind
      // a branch and hipcc waits for each one (one memory round trip per row group)
      v[i] = *(const floatx4*)(xb + (long)(H + min(t0 + r, T - 1) + shift) * 32 + c4);
      if (t0 + r >= T) v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      *(floatx4*)(dst + (e >> 3) * XS + (e & 7) * 4) = v[i];
    }
  } else {
    for (int e = tid; e < LP * 32; e += 256) {
      const int r = e >> 5, c = e & 31;
      float v = 0.f;
      if (t0 + r < T && c < C) v = xb[(long)(H + t0 + r + shift) * C + c];
      dst[r * XS + c] = v;
    }
  }
}

// G[r] = g_a[t] + (t+gd < T ? g_c0[t+gd] : 0) for t = t0 + r (rows of [M][C] buffers of stream b)
LBWN_DEV void stage_g(float* G, const float* __restrict__ ga, const float* __restrict__ gc, int gd, long mb,
                      int t0, int T, int C, int tid) {
  if (!ga) {
    for (int e = tid; e < LP * XS; e += 256) G[e] = 0.f;
    return;
  }
  if (C == 32) {
    floatx4 v[4], u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      const int r = e >> 3, c4 = (e & 7) * 4, t = t0 + r;
      v[i] = *(const floatx4*)(ga + (mb + min(t, T - 1)) * 32 + c4);       // clamped, then select
      u[i] = gc ? *(const floatx4*)(gc + (mb + min(t + gd, T - 1)) * 32 + c4) : floatx4{0.f, 0.f, 0.f, 0.f};
      if (t >= T) v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (t + gd >= T || !gc) u[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      *(floatx4*)(G + (e >> 3) * XS + (e & 7) * 4) = v[i] + u[i];
    }
  } else {
    for (int e = tid; e < LP * 32; e += 256) {
      const int r = e >> 5, c = e & 31, t = t0 + r;
      float v = 0.f;
      if (t < T && c < C) {
        v = ga[(mb + t) * C + c];
        if (gc && t + gd < T) v += gc[(mb + t + gd) * C + c];
      }
      G[r * XS + c] = v;
    }
  }
}

// packed image -> LDS (Ws | Rs | bs | br are contiguous in both)
LBWN_DEV void stage_image(float* W, const float* __restrict__ img, int tid) {
  for (int e = tid; e < WIMG / 4; e += 256) *(floatx4*)(W + 4 * e) = *(const floatx4*)(img + 4 * e);
}

// vᵀ for this wave's 32 positions: acc_s/acc_g rows = out channel, lanes = position.
template <typename K>
LBWN_DEV void conv_tile(const float* Xp, const float* Xc, const float* Ws, const float* bs,
                        const K& a, long m, bool valid, int w, int lane, floatx16& acc_s,
                        floatx16& acc_g) {
  const int pi = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc_s[r] = bs[acc_row(r, h)];
    acc_g[r] = bs[32 + acc_row(r, h)];
  }
  if (valid && (a.gc_tab || a.cond)) {
    const float* cs = a.gc_tab ? a.gc_tab + (long)a.ids[m] * a.gc_ld : nullptr;
    const float* cl = a.cond ? a.cond + m * a.ldcond : nullptr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = acc_row(r, h);
      if (o < a.Cd) {
        if (cs) { acc_s[r] += cs[o]; acc_g[r] += cs[a.Cd + o]; }
        if (cl) { acc_s[r] += cl[o]; acc_g[r] += cl[a.Cd + o]; }
      }
    }
  }
  const float* xp = Xp + (32 * w + pi) * XS;
  const float* xc = Xc + (32 * w + pi) * XS;
  // operands of group g (8 k values: k = 8g+4h+j) are fetched while group g-1's MFMAs issue
  floatx4 bx[2];
  float ws_[2][4], wg_[2][4];
  auto load = [&](int g, int buf) {
    const float* src = g < 4 ? xp : xc;
    bx[buf] = *(const floatx4*)(src + 8 * (g & 3) + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 8 * g + 4 * h + j;
      ws_[buf][j] = Ws[k * WS + pi];
      wg_[buf][j] = Ws[k * WS + 32 + pi];
    }
  };
  load(0, 0);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const int cb = g & 1;
    if (g + 1 < 8) load(g + 1, cb ^ 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc_s = mfma32(ws_[cb][j], bx[cb][j], acc_s);
      acc_g = mfma32(wg_[cb][j], bx[cb][j], acc_g);
    }
  }
}

// σ(v_gate) rows (SG) are stored in 32-row blocks laid out in the MFMA register order, [m/32][q][m%32][h][4]
// (channel 8q + 4h + j), so that each wave-instruction of the forward's stores and of the backward's
// loads covers one contiguous KiB instead of 32 partial lines
LBWN_DEV long sg_off(long m, int q, int h) { return (((m >> 5) * 4 + q) * 32 + (m & 31)) * 8 + 4 * h; }

LBWN_DEV void store_rows16(float* row, const floatx16& v, int C, int h) {
  if (C == 32) {
#pragma unroll
    for (int q = 0; q < 4; ++q) *(floatx4*)(row + 8 * q + 4 * h) = floatx4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (acc_row(r, h) < C) row[acc_row(r, h)] = v[r];
  }
}

// ---- forward ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void layer_fwd_kernel(FwdK a) {
  __shared__ __attribute__((aligned(16))) float sm[2 * LP * XS + WIMG];
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* Ws = Xc + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* br = bs + 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;
  stage_image(Ws, a.wpack, tid);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, t0 = (tile % tps) * LP;
    const float* xb = a.x_in + (long)b * (a.H + a.T) * a.Cr;
    if (tile != (int)blockIdx.x) __syncthreads();  // previous tile's LDS reads done
    stage_rows(Xp, xb, t0, -a.d, a.T, a.H, a.Cr, tid);
    stage_rows(Xc, xb, t0, 0, a.T, a.H, a.Cr, tid);
    __syncthreads();

    const int t = t0 + 32 * w + pi;
    const bool valid = t < a.T;
    const long m = (long)b * a.T + t;
    floatx16 acc_s, acc_g;
    if (LBWN_ABL & 32) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc_s[r] = Xc[r * 8 + lane]; acc_g[r] = Xp[r * 8 + lane]; }
    } else {
      conv_tile(Xp, Xc, Ws, bs, a, m, valid, w, lane, acc_s, acc_g);
    }
    floatx16 z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = tanhf_(acc_s[r]) * sigmoidf_(acc_g[r]);
    if (a.x_out) {
      floatx16 acc_r;
      const float* xc = Xc + (32 * w + pi) * XS;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 xv = *(const floatx4*)(xc + 8 * q + 4 * h);
        const floatx4 bv = *(const floatx4*)(br + 8 * q + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc_r[4 * q + j] = xv[j] + bv[j];
      }
      float ra[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) ra[s] = Rs[acc_row(s, h) * XS + pi];
#pragma unroll
      for (int s = 0; s < 16; ++s) acc_r = mfma32(ra[s], z[s], acc_r);
      if (valid && !(LBWN_ABL & 64)) store_rows16(a.x_out + ((long)b * (a.H + a.T) + a.H + t) * a.Cr, acc_r, a.Cr, h);
      if (LBWN_ABL & 64) asm volatile("" ::"v"(acc_r[0]), "v"(acc_r[15]));
    }
    if (valid && !(LBWN_ABL & 64)) store_rows16(a.z + m * a.ldz, z, a.Cd, h);
    if (LBWN_ABL & 64) asm volatile("" ::"v"(z[0]), "v"(z[15]));
  }
}

// ---- persistent forward chain -------------------------------------------------------------
// The 50 dependent layers as ONE launch.  A block owns a 128-position tile of one stream for
// every layer; its own rows stay in LDS (double-buffered x_l / x_{l+1}), and only the dilated
// tap's halo (rows t0-d .. t0-1: min(d,128) rows of ONE producer tile of the same stream, or
// SAVE) crosses blocks.  Hand-off (cdna_hip_programming §6 G16, R1 form): the producer stores
// x_{l+1} write-through (sc1), every wave drains (s_waitcnt vmcnt(0)), block barrier, one
// lane stores flag[tile] = l+1 (relaxed, agent); the consumer polls that word relaxed from one
// lane, barriers, and reads the halo ONLY with sc1 loads (no acquire fence needed).  The own
// tap (W1·x[t]) is computed before the poll so the hand-off latency hides behind it.
// Deadlock freedom: tiles run in rounds of gridDim.x ≤ resident blocks, in increasing tile
// order; a producer tile is always in the same round (resident) or an earlier one (done).
// Every spin is bounded (SPIN_TIMEOUT) and reports through the status word.
typedef __attribute__((address_space(3))) void lds_void;

// One LDS-DMA piece (global_load_lds_dwordx4: 64 lanes × 16 B from per-lane addresses to
// lds_dst + 16·lane) issued from inline asm, so the compiler neither knows the LDS it writes (no
// conservative vmcnt(0) before every later LDS access) nor counts it: the kernel lands these
// pieces itself with an explicit vmcnt(0) drain + barrier before their first reader.
LBWN_DEV void dma16(const void* g, float* lds_dst) {
  const unsigned base =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds_dst);
  unsigned saved;   // m0 is reserved by the compiler: saved and restored around the piece
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "s"(base), "v"(g)
               : "memory");
}

typedef __attribute__((address_space(1))) unsigned gu32;
constexpr long long SPIN_TIMEOUT = 400000000LL;  // wall_clock64 ticks (100 MHz) = 4 s
constexpr int BUF_DW3 = 0x00020000;

// First tile of this block in the chains' tile walk (tile += gridDim.x after it).  xcd: blocks
// b and b + 8 share an XCD under round-robin dispatch (MI355X_MICROARCH.md, placement: speed only,
// never correctness), so with gridDim.x % 8 == 0 block b takes tile (b % 8)·(G/8) + b / 8 of each
// round: consecutive tiles -- a stream's hand-off neighbours -- run on one XCD (32 tiles = one
// 4096-sample stream at C2).  A bijection of each round's tiles: the rounds are unchanged.
LBWN_DEV int chain_first(int xcd) {
  const int bx = blockIdx.x, G = gridDim.x;
  return (xcd && (G & 7) == 0) ? (bx & 7) * (G >> 3) + (bx >> 3) : bx;
}

struct ChainFK {
  int xcd;                     // chain_first: XCD-grouped tile walk
  float* X; long xls;        // x_l for all layers: layer stride (floats); each [B][H+T][32]
  float* Z; long ldz;
  const float* wpack;        // L packed images
  const float* gc_tab; long gc_ld;              // GC table [ncat+1][L·2Cd] (row stride gc_ld; layer l at l·2Cd)
  const int* ids; const float* cond; long ldcond; // LC term COND [M][L·2Cd] (layer l at column l·2Cd) or null
  unsigned* flags; unsigned* status;
  int B, T, H, L, nbl, Cd;
  long long* trace; int trace_blk;   // debug stamps (null in production)
  const unsigned short* ximg;        // L split images (XIMG_US bf16 each): the bf16-split form
  float* SG; long sgls;              // σ(v_gate) rows [L][M32][32] (sg_off blocks) for chain_bwd_x3_kernel, or null
  // in-chain LC term (chain_fwd_kernel<true, true>): the upsampled LC input [M][Lo] and the L
  // split LC images (LCIMG_US bf16 each)
  const float* lcact; const unsigned short* lcimg; int Lo;
};

// lc·[LC_SIGNAL_l | LC_GATE_l] onto the accumulators (tmodel.py:155-160): A = the layer's LC
// image rows (out channel), B = this lane's LC input row, pre-split once per tile (lcb); the
// fragments of k-step s+1 are read while step s's MFMAs issue
LBWN_DEV void lc_terms(const unsigned short* LI, const bf16x8 (&lcb)[LC_K][3], int pi, int h, floatx16& acc_s,
                       floatx16& acc_g) {
  bf16x8 fs[2][3], fg[2][3];
  auto load = [&](int s2, int buf) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      fs[buf][p] = *(const bf16x8*)(LI + pi * LC_ROW + LC_KP * p + 16 * s2 + 8 * h);
      fg[buf][p] = *(const bf16x8*)(LI + (32 + pi) * LC_ROW + LC_KP * p + 16 * s2 + 8 * h);
    }
  };
  load(0, 0);
#pragma unroll
  for (int s2 = 0; s2 < LC_K; ++s2) {
    const int cb = s2 & 1;
    if (s2 + 1 < LC_K) load(s2 + 1, cb ^ 1);
    acc_s = mfma_x3(fs[cb], lcb[s2], acc_s);
    acc_g = mfma_x3(fg[cb], lcb[s2], acc_g);
  }
}

// one layer's LC image into LDS by LDS-DMA (wave w moves pieces w, w+4, ...); landed by the
// caller's next vmcnt drain + barrier
LBWN_DEV void dma_lc_image(const unsigned short* lcimg, int l, float* LCI, int w, int lane) {
  const float* src = (const float*)lcimg + (long)l * LCIMG_F + lane * 4;
#pragma unroll
  for (int i = 0; i < (LCIMG_F / 256 + 3) / 4; ++i) {
    const int pc = w + 4 * i;
    if (pc < LCIMG_F / 256) dma16(src + pc * 256, LCI + pc * 256);
  }
}

// GC + LC term of layer l for this lane's position, in acc layout: cv[q] = sig channels
// 8q+4h..+3, cv[4+q] = gate channels (16-B loads; issued one layer ahead by the chains).
// CM (compile time): 0 no conditioning, 1 GC only (the in-chain-LC forward of arch5 and GC-only
// archs), 2 any (runtime pointers).  CM 1 loads are issued unconditionally at clamped rows (a row
// past T feeds only its own, discarded, position column) straight into cv: an add right after the
// load (CM 2's zero-init + add) or a register copy merging paths made hipcc wait for the loads --
// with vmcnt(0), which also waited out the x_{l+1} stores issued just before (the drain the own
// tap is meant to hide).
template <int CM, typename K>
LBWN_DEV void load_cond(const K& a, int l, int myid, long m, bool valid, int h, floatx4 (&cv)[8]) {
  if (CM == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) cv[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  if (CM == 1) {
    const float* g = a.gc_tab + (long)myid * a.gc_ld + (long)l * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cv[q] = *(const floatx4*)(g + 8 * q + 4 * h);
      cv[4 + q] = *(const floatx4*)(g + 32 + 8 * q + 4 * h);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) cv[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (!valid) return;
  if (a.gc_tab) {
    const float* g = a.gc_tab + (long)myid * a.gc_ld + (long)l * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cv[q] += *(const floatx4*)(g + 8 * q + 4 * h);
      cv[4 + q] += *(const floatx4*)(g + 32 + 8 * q + 4 * h);
    }
  }
  if (a.cond) {
    const float* c = a.cond + m * a.ldcond + (long)l * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cv[q] += *(const floatx4*)(c + 8 * q + 4 * h);
      cv[4 + q] += *(const floatx4*)(c + 32 + 8 * q + 4 * h);
    }
  }
}

LBWN_DEV bool wait_flag_ge(unsigned* f, unsigned want, unsigned* status, unsigned code) {
  const long long t0 = wall_clock64();
  for (;;) {
    if (__hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
    if (wall_clock64() - t0 > SPIN_TIMEOUT) {
      // OR, not store: the word is zeroed once per step (lbwn_train_forward), so a forward
      // timeout (1) survives the backward chain and both read back as 3
      __hip_atomic_fetch_or((gu32*)status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

LBWN_DEV void publish_flag(unsigned* f, unsigned v) {
  __hip_atomic_store((gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bias + conditioning into the accumulators (acc layout rows = out channel)
LBWN_DEV void conv_init(const float* bs, const floatx4 (&cv)[8], int h, floatx16& acc_s, floatx16& acc_g) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc_s[4 * q + j] = bs[8 * q + 4 * h + j] + cv[q][j];
      acc_g[4 * q + j] = bs[32 + 8 * q + 4 * h + j] + cv[4 + q][j];
    }
}

// acc += Wkᵀ·x over one tap: Wk = the 32 weight-image rows of that tap, xrow = this lane's
// 32-channel input row (LDS)
LBWN_DEV void conv_half(const float* xrow, const float* Wk, int pi, int h, floatx16& acc_s, floatx16& acc_g) {
  // every operand of the 32 MFMAs read first; the sched_barrier stops hipcc from sinking each
  // weight pair next to its MFMA (it did, with an LDS round trip per MFMA pair)
  floatx4 bx[4];
  float ws_[4][4], wg_[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bx[g] = *(const floatx4*)(xrow + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 8 * g + 4 * h + j;
      ws_[g][j] = Wk[k * WS + pi];
      wg_[g][j] = Wk[k * WS + 32 + pi];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc_s = mfma32(ws_[g][j], bx[g][j], acc_s);
      acc_g = mfma32(wg_[g][j], bx[g][j], acc_g);
    }
}

// conv_half on the bf16 cores: acc += Wkᵀ·x over one tap (2 k-steps of 16 channels, sig and
// gate), Wt = the split image's WT at this tap (bf16, rows XW_ROW), x split on the fly
LBWN_DEV void conv_half_x3(const float* xrow, const unsigned short* Wt, int pi, int h, floatx16& acc_s, floatx16& acc_g) {
  floatx4 xv[4];
  bf16x8 ws_[2][3], wg_[2][3];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    xv[2 * c] = *(const floatx4*)(xrow + 16 * c + 8 * h);
    xv[2 * c + 1] = *(const floatx4*)(xrow + 16 * c + 8 * h + 4);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      ws_[c][p] = *(const bf16x8*)(Wt + pi * XW_ROW + 32 * p + 16 * c + 8 * h);
      wg_[c][p] = *(const bf16x8*)(Wt + (32 + pi) * XW_ROW + 32 * p + 16 * c + 8 * h);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    bf16x8 xb[3];
    split8(xv[2 * c], xv[2 * c + 1], xb);
    acc_s = mfma_x3(ws_[c], xb, acc_s);
    acc_g = mfma_x3(wg_[c], xb, acc_g);
  }
}

static_assert(4096 + 768 <= 2 * LP * XS, "RED + bias partials must fit in Xp and Xc");
constexpr int CF_LDS = 3 * LP * XS + 2 * WIMG;      // Xc[2] | HALO | IMG[2]  (99.8 KB)
constexpr int IMG_PF = (WIMG / 4 + 255) / 256;      // float4 per thread to prefetch an image
constexpr int CF_LDS_X3 = 3 * LP * XS + 2 * XIMG_F;  // with split images (120.6 KB)
constexpr int CF_LDS_X3LC = CF_LDS_X3 + LCIMG_F;      // + one LC image (151.6 KB)
static_assert(CF_LDS_X3LC * 4 + 16 <= 160 * 1024, "chain fwd x3 + LC LDS");

// Per layer l (weight image IMG[l&1]):
//   wait for the producer tile's x_l, halo rows (sc1 loads), barrier;
//   dilated tap W0·x[t-d] onto the accumulators that already hold W1·x[t] (done last layer);
//   gate; residual → x_{l+1} to LDS and (sc1) to HBM;
//   the NEXT layer's own tap W1'·x_{l+1}[t]: it reads only rows this wave just wrote, so it needs
//   no barrier and runs while the x stores drain; then drain, barrier, publish, z store, and
//   the image of layer l+2 into IMG[l&1] (dead after that barrier; first read after the next
//   layer's halo barrier).  Double-buffered images are what let the own tap move: one image
//   forced a barrier between this layer's last read and the next layer's first.
// X3: the conv and residual products on the bf16 cores from split images (ChainFK::ximg);
// otherwise v_mfma_f32_32x32x2_f32 from the f32 images.
// LC (X3 only): the LC term lc·LC_l computed in the chain (no [M][L·2Cd] COND round trip): the
// tile's LC input rows are split once into registers; the layer's LC image (one LDS buffer) is
// read with the own tap in step 7 of the previous layer (tile start for layer 0), and the image
// two layers ahead is LDS-DMA'd in step 9, after the publish barrier (every wave is past its
// reads), landing with the next layer's halo loads (in-order vmcnt) before its halo barrier.
// TR: the traced build (in-kernel clock stamps, lbwn_plan's LBWN_CHAIN_TRACE): the stamps'
// lane-divergent branches cost the untraced chains 0.5-3 % (same-box A/B, tools/ab_step.sh)
template <bool X3, bool LC, int CM, bool TR>
__global__ __launch_bounds__(256) void chain_fwd_kernel(ChainFK a) {
  static_assert(X3 || !LC, "in-chain LC needs the split images");
  constexpr int IMGF = X3 ? XIMG_F : WIMG;              // floats per layer image
  constexpr int PF = (IMGF / 4 + 255) / 256;            // float4 per thread to prefetch one
  __shared__ __attribute__((aligned(16))) float sm[LC ? CF_LDS_X3LC : X3 ? CF_LDS_X3 : CF_LDS];
  __shared__ int s_fail;
  float* HALO = sm + 2 * LP * XS;
  float* IMG0 = HALO + LP * XS;
  // f32: [W 64×WS | R 32×XS | bs 64 | br 32]; X3: [WT | RT | bs 64 | br 32] (bf16 + f32)
  auto img = [&](int l) { return IMG0 + (l & 1) * IMGF; };
  float* LCI = IMG0 + 2 * IMGF;   // LC: the one LC image buffer
  const unsigned short* LCIu = (const unsigned short*)LCI;
  const float* wsrc = X3 ? (const float*)a.ximg : a.wpack;
  auto bias_of = [&](const float* im) { return X3 ? im + XB_OFF / 2 : im + 64 * WS + 32 * XS; };

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int r = 32 * w + pi;  // this lane's row of the tile
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;
  if (tid == 0) s_fail = 0;
  const int first = chain_first(a.xcd);
  for (int tile = first; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, tt = tile % tps, t0 = tt * LP;
    const int t = t0 + r;
    const bool valid = t < a.T;
    const long m = (long)b * a.T + t;
    const long sb = (long)b * (a.H + a.T) * 32;  // stream base inside a layer buffer
    constexpr bool has_cond = CM != 0;
    const int myid = (a.gc_tab && valid) ? a.ids[m] : 0;
    floatx4 cv[8];
    load_cond<CM>(a, 0, myid, m, valid && has_cond, h, cv);
    // LC: this lane's LC input row, split once for the tile (B operand: k = 16s + 8h + j)
    bf16x8 lcb[LC_K][3];
    if (LC) {
      const float* lrow = a.lcact + ((long)b * a.T + min(t, a.T - 1)) * a.Lo;
#pragma unroll
      for (int s2 = 0; s2 < LC_K; ++s2) {
        const int k0 = 16 * s2 + 8 * h;
        floatx4 u = *(const floatx4*)(lrow + min(k0, a.Lo - 4));       // clamped, then select
        floatx4 v = *(const floatx4*)(lrow + min(k0 + 4, a.Lo - 4));
        if (k0 >= a.Lo) u = floatx4{0.f, 0.f, 0.f, 0.f};
        if (k0 + 4 >= a.Lo) v = floatx4{0.f, 0.f, 0.f, 0.f};
        split8(u, v, lcb[s2]);
      }
    }
    __syncthreads();  // previous tile's LDS use done
    if (LC) dma_lc_image(a.lcimg, 0, LCI, w, lane);
    {  // images of layers 0 and 1 (contiguous in both places): every load issued before the first
       // store (a load-store loop waited out one round trip per iteration)
      constexpr int NI = (2 * IMGF / 4 + 255) / 256;
      const int nimg4 = min(a.L, 2) * IMGF / 4;
      floatx4 iv[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) iv[i] = *(const floatx4*)(wsrc + 4 * min(tid + 256 * i, nimg4 - 1));
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int e = tid + 256 * i;
        if (e < nimg4) *(floatx4*)(img(0) + 4 * e) = iv[i];
      }
    }
    stage_rows(sm, a.X + sb, t0, 0, a.T, a.H, 32, tid);  // x_0 (embed output, pre-launch)
    if (LC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the LC image DMA
    __syncthreads();
    // layer 0's own tap W1·x_0[t] (+ its LC term)
    floatx16 acc_s, acc_g;
    conv_init(bias_of(img(0)), cv, h, acc_s, acc_g);
    if (has_cond && a.L > 1) load_cond<CM>(a, 1, myid, m, valid, h, cv);
    if (X3) conv_half_x3(sm + r * XS, (const unsigned short*)img(0) + 96, pi, h, acc_s, acc_g);
    else conv_half(sm + r * XS, img(0) + 32 * WS, pi, h, acc_s, acc_g);
    if (LC) {
      lc_terms(LCIu, lcb, pi, h, acc_s, acc_g);
      if (a.L > 1) {
        __syncthreads();   // every wave is past its LC_0 reads
        dma_lc_image(a.lcimg, 1, LCI, w, lane);   // lands with layer 0's halo loads
      }
    }
    const bool trc = a.trace && (int)blockIdx.x == a.trace_blk && tid == 0 && tile == first;
#define FSTAMP(i) if (TR && trc) a.trace[16 * l + (i)] = clock64()
    auto store_zs = [&](int ll, const floatx16& zz, const floatx16& ss) {
      if (valid) store_rows16(a.Z + m * a.ldz + (long)ll * a.Cd, zz, a.Cd, h);
      if (X3 && a.SG && valid) {
        float* sgl = a.SG + (long)ll * a.sgls;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *(floatx4*)(sgl + sg_off(m, q, h)) = floatx4{ss[4 * q], ss[4 * q + 1], ss[4 * q + 2], ss[4 * q + 3]};
      }
    };
    for (int l = 0; l < a.L; ++l) {
      FSTAMP(0);
      const int d = 1 << (l % a.nbl);
      float* cur = sm + (l & 1) * LP * XS;
      float* nxt = sm + ((l + 1) & 1) * LP * XS;
      float* xl = a.X + (long)l * a.xls + sb;
      const float* Wl = img(l);
      const float* Rs = Wl + 64 * WS;
      const float* br = bias_of(Wl) + 64;
      floatx4 pf[PF];   // image of layer l+2, loaded in step 3
      FSTAMP(1);
      // 2. wait for the producer of the halo rows (x_l is layer l-1's output)
      const int ptt = tt - max(1, d / LP);
      if (l > 0 && ptt >= 0) {
        if (tid == 0 && !s_fail) {
          if (!wait_flag_ge(a.flags + (long)b * tps + ptt, (unsigned)l, a.status, 1u)) s_fail = 1;
        }
        __syncthreads();
      }
      FSTAMP(2);
      // 3. halo rows [0, min(d,LP)): x_l rows t0-d+row (SAVE rows when < 0), sc1 loads
      {
        const int nh = min(d, LP);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(xl, (short)0, (int)((long)(a.H + a.T) * 32 * 4), BUF_DW3);
        floatx4 hv[4];   // all four issued before the first is stored (clamped rows)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = min(tid + 256 * i, nh * 8 - 1), row = e >> 3, c4 = (e & 7) * 4;
          hv[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((a.H + t0 + row - d) * 32 + c4) * 4, 0, 16);
        }
        // 1. prefetch the image of layer l+2 (pre-launch data: plain loads, clamped: no branch),
        //    issued BEHIND the halo loads: the halo wait then leaves them in flight (vmcnt(PF)),
        //    where in front of the producer poll they were waited out by lane 0's vmcnt(0)
        //    (unconditional, at a clamped layer: a skipped branch made hipcc wait as if they were
        //    not in flight)
        {
          const floatx4* src = (const floatx4*)(wsrc + (long)min(l + 2, a.L - 1) * IMGF);
#pragma unroll
          for (int i = 0; i < PF; ++i) pf[i] = src[min(tid + 256 * i, IMGF / 4 - 1)];
        }
        // every HALO row written (rows >= nh get a copy of row nh-1 and are never read: only rows
        // r < d are): a store behind `e < nh*8` made hipcc sink the 4th load into that branch,
        // issued after the first three had drained (one more L2 round trip per layer)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = tid + 256 * i;
          *(floatx4*)(HALO + (e >> 3) * XS + (e & 7) * 4) = hv[i];
        }
      }
      __syncthreads();
      FSTAMP(3);
      // 4. residual weights read now (they wait behind the conv, not in front of the residual)
      float ra[16];
      bf16x8 rf[2][3];   // X3: RT fragments of the two 16-channel k-steps
      if (X3) {
        const unsigned short* rt = (const unsigned short*)Wl + 64 * XW_ROW + pi * XR_ROW + 8 * h;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int p = 0; p < 3; ++p) rf[s2][p] = *(const bf16x8*)(rt + 32 * p + 16 * s2);
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) ra[s2] = Rs[acc_row(s2, h) * XS + pi];
      }
      __builtin_amdgcn_sched_barrier(0);
      // 5. dilated tap W0·x[t-d], gate
      const float* xp = (r >= d) ? cur + (r - d) * XS : HALO + r * XS;
      if (X3) conv_half_x3(xp, (const unsigned short*)Wl, pi, h, acc_s, acc_g);
      else conv_half(xp, Wl, pi, h, acc_s, acc_g);
      floatx16 z, sgv;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float sq;
        z[q] = gate_zs(acc_s[q], acc_g[q], sq);
        sgv[q] = sq;
      }
      FSTAMP(4);
      if (l + 1 < a.L) {
        // 6. residual: x_{l+1} = x_l + br + RES·z → LDS (next layer's rows) and HBM (sc1)
        floatx16 acc_r;
        const float* xc = cur + r * XS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 xv = *(const floatx4*)(xc + 8 * q + 4 * h);
          const floatx4 bv = *(const floatx4*)(br + 8 * q + 4 * h);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc_r[4 * q + j] = xv[j] + bv[j];
        }
        if (X3) {
          // z (acc layout) is the B operand: registers 8s..8s+7 form k-step s (RT holds the
          // matching permuted channel order)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            bf16x8 zb[3];
            split8(floatx4{z[8 * s2], z[8 * s2 + 1], z[8 * s2 + 2], z[8 * s2 + 3]},
                   floatx4{z[8 * s2 + 4], z[8 * s2 + 5], z[8 * s2 + 6], z[8 * s2 + 7]}, zb);
            acc_r = mfma_x3(rf[s2], zb, acc_r);
          }
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) acc_r = mfma32(ra[s2], z[s2], acc_r);
        }
        float* xn = a.X + (long)(l + 1) * a.xls + sb;
        const __amdgpu_buffer_rsrc_t rn =
            __builtin_amdgcn_make_buffer_rsrc(xn, (short)0, (int)((long)(a.H + a.T) * 32 * 4), BUF_DW3);
        float* nrow = nxt + r * XS;
        // only the rows the next layer's consumer tile reads (the last min(d_{l+1}, LP)) cross
        // CUs inside this launch: those are written through (sc1) and drained before the publish;
        // the rest are plain stores, read after the launch (backward, SAVE).  Writing every row
        // through cost ~3k cycles per layer (drain 2.4k + slower issue; tools/fwd_abl.sh)
        const bool halo_row = r >= LP - min(1 << ((l + 1) % a.nbl), LP);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 v = floatx4{acc_r[4 * q], acc_r[4 * q + 1], acc_r[4 * q + 2], acc_r[4 * q + 3]};
          *(floatx4*)(nrow + 8 * q + 4 * h) = v;
          const int off = ((a.H + t) * 32 + 8 * q + 4 * h) * 4;
          if (valid && halo_row) __builtin_amdgcn_raw_buffer_store_b128(v, rn, off, 0, 16);
          if (valid && !halo_row) __builtin_amdgcn_raw_buffer_store_b128(v, rn, off, 0, 0);
        }
        FSTAMP(8);
        // 7. the next layer's own tap from the row this wave just wrote (wave-local: no barrier)
        //    while the x stores drain; its image IMG[(l+1)&1] landed before this layer's barriers
        wave_lds_fence();
        const float* Wn = img(l + 1);
        conv_init(bias_of(Wn), cv, h, acc_s, acc_g);
        if (has_cond && l + 2 < a.L) load_cond<CM>(a, l + 2, myid, m, valid, h, cv);
        if (X3) conv_half_x3(nrow, (const unsigned short*)Wn + 96, pi, h, acc_s, acc_g);
        else conv_half(nrow, Wn + 32 * WS, pi, h, acc_s, acc_g);
        if (LC) lc_terms(LCIu, lcb, pi, h, acc_s, acc_g);   // LC_{l+1}: landed before this layer's halo barrier
      }
      FSTAMP(5);
      // 8. publish x_{l+1}: every wave drains its sc1 stores, barrier, one lane signals
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      FSTAMP(9);
      __syncthreads();
      FSTAMP(10);
      if (tid == 0 && l + 1 < a.L) publish_flag(a.flags + tile, (unsigned)(l + 1));
      // 9. image of layer l+2 into IMG[l&1] (everyone is past this layer's reads of it; its loads
      //    landed with the drain), and the LC image of layer l+2 (LC_{l+1} was read in step 7,
      //    before the publish barrier)
      if (LC && l + 2 < a.L) dma_lc_image(a.lcimg, l + 2, LCI, w, lane);
      if (l + 2 < a.L) {
        float* dst = IMG0 + (l & 1) * IMGF;
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const int e = tid + 256 * i;
          if (e < IMGF / 4) *(floatx4*)(dst + 4 * e) = pf[i];
        }
      }
      FSTAMP(6);
      // 10. z (skip GEMM input) and σ rows, issued last: they drain in the shadow of the next
      //     layer (written before the image, the image writes' vmcnt waits waited them out)
      // (stored during the next layer instead, after its halo barrier, they lengthened that
      // layer's publish drain: forward 276 -> 287 us, same box)
      store_zs(l, z, sgv);
      FSTAMP(7);
    }
#undef FSTAMP
  }
}

// ---- forward chain, 16-position waves (round 4) ---------------------------------------------
// chain_fwd16_kernel<NW, LC, CM, TR>: the X3 forward chain on v_mfma_f32_16x16x32_bf16 with 16
// positions per wave and NW waves per block: tile TP = 16·NW positions (the C4 tile axis:
// NW = 8 → 128 positions with TWO waves per SIMD, NW = 4 → 64 positions).  The per-layer protocol
// (halo hand-off, own tap of the next layer inside the store drain, double-buffered images, the
// LC image two layers ahead) is chain_fwd_kernel's; what changes is the MFMA geometry:
//   lane = (j = lane & 15: the wave's position, g = lane >> 4), and with q0 = 2(g >> 1), h = g & 1
//   the lane's accumulator block b (0, 1) register r holds channel 8(q0 + b) + 4h + r — the same
//   (q, h) channel groups chain_fwd_kernel's lanes hold, so z / σ go to the same rows / sg_off
//   blocks and the residual's B operand (the lane's 8 z values) is in the split image's RT k order
//   unchanged.  For that, conv A row i of block b reads out channel ch16(b, i) (the permutation
//   that puts D row i = 4g + r on that channel).  The residual's rows are unpermuted: x_{l+1}
//   block rb register r = channel 16rb + 4g + r.
// Per wave and layer: conv 2 taps × (sig, gate) × 2 blocks × 6 products = 48 MFMAs of 16 cycles,
// residual 2 blocks × 6 = 12 — per position the MFMA work of chain_fwd_kernel, in half the
// positions per wave, so two waves share each SIMD at NW = 8 and hide each other's latencies.
LBWN_DEV int ch16(int b, int i) { return 16 * (i >> 3) + 8 * b + 4 * ((i >> 2) & 1) + (i & 3); }

// acc += A·B over one 32-deep k-step from split fragments (six products, small terms first)
LBWN_DEV floatx4 mfma16x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// LC image of the 16-lane form: LCT16[o (sig 0..31 | gate 32..63)][plane][k 0..95] (k >= n_lc_out
// zero: three whole 32-deep k-steps), rows of LC16_ROW = 3·96 + 8 bf16 (148 dwords: 4·odd).
constexpr int LC16_KP = 96, LC16_ROW = 3 * LC16_KP + 8;
constexpr int LC16IMG_US = 64 * LC16_ROW;                      // bf16 elements per layer image
constexpr int LC16IMG_F = LC16IMG_US / 2;                      // = 9472 floats = 37 KiB
static_assert(LC16IMG_F % 256 == 0, "LC16 image: whole 1-KiB DMA pieces");

LBWN_DEV void pack_lc16_body(int l, const float* lsig, const float* lgate, unsigned short* out, int Lo, int Cd) {
  unsigned short* img = out + (long)l * LC16IMG_US;
  for (int e = threadIdx.x; e < 64 * (LC16_ROW / 2); e += blockDim.x) {
    const int o = e / (LC16_ROW / 2), kk = 2 * (e % (LC16_ROW / 2));
    unsigned short* row = img + o * LC16_ROW;
    if (kk >= LC16_KP) {   // row pad (zero); plane slots are written below
      if (kk >= 3 * LC16_KP) *(unsigned*)(row + kk) = 0u;
      continue;
    }
    const float* w = (o < 32 ? lsig : lgate) + (long)l * Lo * Cd;
    const int oc = o & 31;
    floatx2 x = {0.f, 0.f};
    if (oc < Cd) {
      if (kk < Lo) x[0] = w[(long)kk * Cd + oc];
      if (kk + 1 < Lo) x[1] = w[(long)(kk + 1) * Cd + oc];
    }
    unsigned hi, mi, lo;
    split2(x, hi, mi, lo);
    *(unsigned*)(row + kk) = hi;
    *(unsigned*)(row + LC16_KP + kk) = mi;
    *(unsigned*)(row + 2 * LC16_KP + kk) = lo;
  }
}

template <int NW>
LBWN_DEV void dma_lc16_image(const unsigned short* lcimg, int l, float* LCI, int w, int lane) {
  const float* src = (const float*)lcimg + (long)l * LC16IMG_F + lane * 4;
  constexpr int NP = LC16IMG_F / 256;
#pragma unroll
  for (int i = 0; i < (NP + NW - 1) / NW; ++i) {
    const int pc = w + NW * i;
    if (pc < NP) dma16(src + pc * 256, LCI + pc * 256);
  }
}

// GC / COND term of layer l for this lane's channels: cv[2·kind + b] = channels 8(q0+b)+4h..+3
// (kind 0 sig, 1 gate); CM as load_cond
template <int CM>
LBWN_DEV void load_cond16(const ChainFK& a, int l, int myid, long m, bool valid, int q0, int h, floatx4 (&cv)[4]) {
  if (CM == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) cv[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  if (CM == 1) {
    const float* g = a.gc_tab + (long)myid * a.gc_ld + (long)l * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) cv[i] = *(const floatx4*)(g + 32 * (i >> 1) + 8 * (q0 + (i & 1)) + 4 * h);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) cv[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (!valid) return;
  if (a.gc_tab) {
    const float* g = a.gc_tab + (long)myid * a.gc_ld + (long)l * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) cv[i] += *(const floatx4*)(g + 32 * (i >> 1) + 8 * (q0 + (i & 1)) + 4 * h);
  }
  if (a.cond) {
    const float* c = a.cond + m * a.ldcond + (long)l * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) cv[i] += *(const floatx4*)(c + 32 * (i >> 1) + 8 * (q0 + (i & 1)) + 4 * h);
  }
}

// acc[2·kind + b] = bias + conditioning
LBWN_DEV void conv16_init(const float* bs, const floatx4 (&cv)[4], int q0, int h, floatx4 (&acc)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const floatx4 bv = *(const floatx4*)(bs + 32 * (i >> 1) + 8 * (q0 + (i & 1)) + 4 * h);
    acc[i] = bv + cv[i];
  }
}

// acc += Wtapᵀ·x for one tap: Wt = the split image's WT at this tap (rows XW_ROW), xrow = this
// lane's position row in LDS (channels 8g..8g+7 = the B operand's k group); the operands of each
// of the NP parts (4 / NP accumulator blocks) are read before its MFMAs (NP = 2 halves the live
// fragments for the register-tight LC form)
template <int NP = 1>
LBWN_DEV void conv16_tap_x(floatx4 x0, floatx4 x1, const unsigned short* Wt, int i16, int g, floatx4 (&acc)[4]) {
  bf16x8 xb[3];
#pragma unroll
  for (int part = 0; part < NP; ++part) {
    constexpr int NB = 4 / NP;
    bf16x8 wf[NB][3];
#pragma unroll
    for (int ii = 0; ii < NB; ++ii) {
      const int i = part * NB + ii, o = 32 * (i >> 1) + ch16(i & 1, i16);
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[ii][p] = *(const bf16x8*)(Wt + o * XW_ROW + 32 * p + 8 * g);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (part == 0) split8(x0, x1, xb);
#pragma unroll
    for (int ii = 0; ii < NB; ++ii) acc[part * NB + ii] = mfma16x3(wf[ii], xb, acc[part * NB + ii]);
  }
}
template <int NP = 1>
LBWN_DEV void conv16_tap(const float* xrow, const unsigned short* Wt, int i16, int g, floatx4 (&acc)[4]) {
  conv16_tap_x<NP>(*(const floatx4*)(xrow + 8 * g), *(const floatx4*)(xrow + 8 * g + 4), Wt, i16, g, acc);
}

// lc·[LC_SIGNAL_l | LC_GATE_l] onto the accumulators: A = LC16 image rows, B = the lane's LC input
// row (k = 32s + 8g + j), held as raw f32 (lcv: 24 registers instead of 36 pre-split: at two
// waves per SIMD the split form spilled) and split per k-step
LBWN_DEV void lc16_terms(const unsigned short* LI, const floatx4 (&lcv)[6], int i16, int g, floatx4 (&acc)[4]) {
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    bf16x8 xb[3];
    split8(lcv[2 * s2], lcv[2 * s2 + 1], xb);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 32 * (i >> 1) + ch16(i & 1, i16);
      bf16x8 wf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[p] = *(const bf16x8*)(LI + o * LC16_ROW + LC16_KP * p + 32 * s2 + 8 * g);
      acc[i] = mfma16x3(wf, xb, acc[i]);
    }
  }
}

template <int NW>
constexpr int cf16_lds(bool lc) { return 3 * 16 * NW * XS + 2 * XIMG_F + (lc ? LC16IMG_F : 0); }
static_assert(cf16_lds<8>(true) * 4 + 16 <= 160 * 1024, "chain fwd16 + LC LDS");

template <int NW, bool LC, int CM, bool TR>
__global__ __launch_bounds__(64 * NW) void chain_fwd16_kernel(ChainFK a) {
  constexpr int TP = 16 * NW, NT = 64 * NW;
  constexpr int IMGF = XIMG_F;
  // the LC form (register-tight at two waves per SIMD) moves the image of layer l+2 by LDS-DMA
  // after the publish barrier (landing with the next layer's halo loads, like the LC image);
  // the others prefetch it into registers behind the halo loads and write it after the barrier
  constexpr bool DMAIMG = LC;
  // per-wave halo (below)
  constexpr bool WH = true;
  // LC form: the LC term of layer l+1 (72 MFMAs per wave) runs after layer l's publish instead of
  // inside its store drain, where it outlasted the drain and held the publish back; its image is
  // DMA'd during layer l (after the dilated tap: ahead of the halo loads it would have held their
  // vmcnt waits) into the single LCI buffer, which nothing reads between layer l's top barrier and
  // its publish barrier
  constexpr bool LCLATE = LC;
  constexpr int PF = DMAIMG ? 1 : (IMGF / 4 + NT - 1) / NT;   // float4 per thread to prefetch one image
  constexpr int NR = TP * 8 / NT;                       // float4 per thread of a TP-row tile (2)
  __shared__ __attribute__((aligned(16))) float sm[cf16_lds<NW>(LC)];
  __shared__ int s_fail;
  float* HALO = sm + 2 * TP * XS;
  float* IMG0 = HALO + TP * XS;
  auto img = [&](int l) { return IMG0 + (l & 1) * IMGF; };
  float* LCI = IMG0 + 2 * IMGF;
  const unsigned short* LCIu = (const unsigned short*)LCI;
  const float* wsrc = (const float*)a.ximg;
  auto bias_of = [&](const float* im) { return im + XB_OFF / 2; };

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4, q0 = 2 * (g >> 1), h = g & 1;
  const int r = 16 * w + i16;  // this lane's row of the tile
  const int tps = (a.T + TP - 1) / TP, ntiles = a.B * tps;
  if (tid == 0) s_fail = 0;
  const int first = chain_first(a.xcd);
  for (int tile = first; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, tt = tile % tps, t0 = tt * TP;
    const int t = t0 + r;
    const bool valid = t < a.T;
    const long m = (long)b * a.T + t;
    const long sb = (long)b * (a.H + a.T) * 32;
    constexpr bool has_cond = CM != 0;
    const int myid = (a.gc_tab && valid) ? a.ids[m] : 0;
    floatx4 cv[4];
    load_cond16<CM>(a, 0, myid, m, valid && has_cond, q0, h, cv);
    floatx4 lcv[6];   // LC: this lane's LC input row, k = 32s + 8g + 0..7 (zero past n_lc_out)
    if (LC) {
      const float* lrow = a.lcact + ((long)b * a.T + min(t, a.T - 1)) * a.Lo;
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int k0 = 32 * s2 + 8 * g;
        lcv[2 * s2] = *(const floatx4*)(lrow + min(k0, a.Lo - 4));       // clamped, then select
        lcv[2 * s2 + 1] = *(const floatx4*)(lrow + min(k0 + 4, a.Lo - 4));
        if (k0 >= a.Lo) lcv[2 * s2] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (k0 + 4 >= a.Lo) lcv[2 * s2 + 1] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
    __syncthreads();  // previous tile's LDS use done
    if (LC) dma_lc16_image<NW>(a.lcimg, 0, LCI, w, lane);
    {  // images of layers 0 and 1, every load before the first store
      constexpr int NI = (2 * IMGF / 4 + NT - 1) / NT;
      const int nimg4 = min(a.L, 2) * IMGF / 4;
      floatx4 iv[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) iv[i] = *(const floatx4*)(wsrc + 4 * min(tid + NT * i, nimg4 - 1));
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int e = tid + NT * i;
        if (e < nimg4) *(floatx4*)(img(0) + 4 * e) = iv[i];
      }
    }
    {  // x_0 rows (embed output, pre-launch): unconditional clamped loads, then select
      const float* xb = a.X + sb;
      floatx4 v[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int e = tid + NT * i, rr = e >> 3, c4 = (e & 7) * 4;
        v[i] = *(const floatx4*)(xb + (long)(a.H + min(t0 + rr, a.T - 1)) * 32 + c4);
        if (t0 + rr >= a.T) v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int e = tid + NT * i;
        *(floatx4*)(sm + (e >> 3) * XS + (e & 7) * 4) = v[i];
      }
    }
    if (LC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the LC image DMA
    __syncthreads();
    // layer 0's own tap W1·x_0[t] (+ its LC term)
    floatx4 acc[4];
    conv16_init(bias_of(img(0)), cv, q0, h, acc);
    if (has_cond && a.L > 1) load_cond16<CM>(a, 1, myid, m, valid, q0, h, cv);
    conv16_tap<LC ? 2 : 1>(sm + r * XS, (const unsigned short*)img(0) + 96, i16, g, acc);
    if (LC) {
      lc16_terms(LCIu, lcv, i16, g, acc);
      if (a.L > 1) {
        __syncthreads();   // every wave is past its LC_0 reads
        dma_lc16_image<NW>(a.lcimg, 1, LCI, w, lane);   // lands with layer 0's halo loads
      }
    }
    const bool trc = a.trace && (int)blockIdx.x == a.trace_blk && tid == 0 && tile == first;
#define FSTAMP(i) if (TR && trc) a.trace[16 * l + (i)] = clock64()
    for (int l = 0; l < a.L; ++l) {
      FSTAMP(0);
      const int d = 1 << (l % a.nbl);
      float* cur = sm + (l & 1) * TP * XS;
      float* nxt = sm + ((l + 1) & 1) * TP * XS;
      float* xl = a.X + (long)l * a.xls + sb;
      const float* Wl = img(l);
      const float* br = bias_of(Wl) + 64;
      floatx4 pf[PF];
      FSTAMP(1);
      const int ptt = tt - max(1, d / TP);
      floatx4 hx[2];   // WH: this lane's halo row x[t0 + r - d], channels 8g..8g+7 (rows r < d)
      // (zeroed in the LC form: left undefined on the waves that do not load it, the registers
      // stayed live around the loop there and spilled; zeroed in the others, C2's forward measured
      // 206 -> 216 us)
      if (LC) hx[0] = hx[1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (WH) {
        // per-wave halo: only the waves holding rows r < d wait for the producer (one lane polls)
        // and load their lanes' halo rows into registers; the rest start the layer at once, so a
        // SIMD's other wave computes through the hand-off.  The barrier here only publishes the
        // image written after the last layer's end barrier (the own tap of the next layer reads it
        // before any later barrier)
        // (DMAIMG: the images of layer l+1 DMA'd at the end of the last layer land first)
        if (DMAIMG && l > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l > 0) __syncthreads();
        FSTAMP(2);
        const int nh = min(d, TP);
        if (16 * w < nh) {
          if (l > 0 && ptt >= 0 && lane == 0 && !s_fail) {
            if (!wait_flag_ge(a.flags + (long)b * tps + ptt, (unsigned)l, a.status, 1u)) s_fail = 1;
          }
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(xl, (short)0, (int)((long)(a.H + a.T) * 32 * 4), BUF_DW3);
          const int off = ((a.H + t0 + min(r, nh - 1) - d) * 32 + 8 * g) * 4;
          hx[0] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
          hx[1] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 16);
        }
        if (!DMAIMG) {   // the image of layer l+2 behind the halo loads
          const floatx4* src = (const floatx4*)(wsrc + (long)min(l + 2, a.L - 1) * IMGF);
#pragma unroll
          for (int i = 0; i < PF; ++i) pf[i] = src[min(tid + NT * i, IMGF / 4 - 1)];
        }
      } else {
      // wait for the producer of the halo rows
      if (l > 0 && ptt >= 0) {
        if (tid == 0 && !s_fail) {
          if (!wait_flag_ge(a.flags + (long)b * tps + ptt, (unsigned)l, a.status, 1u)) s_fail = 1;
        }
        __syncthreads();
      }
      FSTAMP(2);
      {  // halo rows [0, min(d,TP)): sc1 loads (clamped rows), then the image of layer l+2 behind them
        const int nh = min(d, TP);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(xl, (short)0, (int)((long)(a.H + a.T) * 32 * 4), BUF_DW3);
        floatx4 hv[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int e = min(tid + NT * i, nh * 8 - 1), row = e >> 3, c4 = (e & 7) * 4;
          hv[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((a.H + t0 + row - d) * 32 + c4) * 4, 0, 16);
        }
        if (!DMAIMG) {
          const floatx4* src = (const floatx4*)(wsrc + (long)min(l + 2, a.L - 1) * IMGF);
#pragma unroll
          for (int i = 0; i < PF; ++i) pf[i] = src[min(tid + NT * i, IMGF / 4 - 1)];
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int e = tid + NT * i;
          *(floatx4*)(HALO + (e >> 3) * XS + (e & 7) * 4) = hv[i];
        }
      }
      __syncthreads();
      }
      FSTAMP(3);
      // residual weights (RT rows 16rb + i16, k group g) read now
      // (the LC form, register-tight, reads them after the dilated tap: with the halo row in
      // registers across them it spilled)
      bf16x8 rf[2][3];
      auto read_rf = [&]() {
        const unsigned short* rt = (const unsigned short*)Wl + 64 * XW_ROW + i16 * XR_ROW + 8 * g;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int p = 0; p < 3; ++p) rf[rb][p] = *(const bf16x8*)(rt + 16 * rb * XR_ROW + 32 * p);
      };
      if (!LC) read_rf();
      __builtin_amdgcn_sched_barrier(0);
      // dilated tap W0·x[t-d], gate
      if (WH) {
        const float* xp = cur + max(r - d, 0) * XS + 8 * g;
        floatx4 x0 = *(const floatx4*)xp, x1 = *(const floatx4*)(xp + 4);
        if (r < d) {
          x0 = hx[0];
          x1 = hx[1];
        }
        conv16_tap_x<LC ? 2 : 1>(x0, x1, (const unsigned short*)Wl, i16, g, acc);
        if (LC) read_rf();
        if (LCLATE && l > 0 && l + 1 < a.L) dma_lc16_image<NW>(a.lcimg, l + 1, LCI, w, lane);
      } else {
        const float* xp = (r >= d) ? cur + (r - d) * XS : HALO + r * XS;
        conv16_tap<LC ? 2 : 1>(xp, (const unsigned short*)Wl, i16, g, acc);
      }
      floatx4 z[2], sg[2];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float sq;
          z[bb][j] = gate_zs(acc[bb][j], acc[2 + bb][j], sq);
          sg[bb][j] = sq;
        }
      // z (skip GEMM input) and σ rows (sg_off blocks for chain_bwd_x3_kernel): issued last, after
      // the publish, so the drain before it does not wait for them -- except in the LC form, whose
      // 16 registers they hold through the residual and the next own tap spilled with the
      // per-wave halo
      auto store_zs = [&]() {
        if (valid) {
          float* zr = a.Z + m * a.ldz + (long)l * a.Cd;
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) *(floatx4*)(zr + 8 * (q0 + bb) + 4 * h) = z[bb];
          if (a.SG) {
            float* sgl = a.SG + (long)l * a.sgls;
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) *(floatx4*)(sgl + sg_off(m, q0 + bb, h)) = sg[bb];
          }
        }
      };
      if (LC) store_zs();
      FSTAMP(4);
      if (l + 1 < a.L) {
        // residual: x_{l+1} = x_l + br + RES·z → LDS (next layer's rows) and HBM (sc1 for halo rows)
        floatx4 accr[2];
        const float* xc = cur + r * XS;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          accr[rb] = *(const floatx4*)(xc + 16 * rb + 4 * g) + *(const floatx4*)(br + 16 * rb + 4 * g);
        {
          bf16x8 zb[3];
          split8(z[0], z[1], zb);   // k = 8g + j: block 0 regs, then block 1 regs (RT's k order)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) accr[rb] = mfma16x3(rf[rb], zb, accr[rb]);
        }
        float* xn = a.X + (long)(l + 1) * a.xls + sb;
        const __amdgpu_buffer_rsrc_t rn =
            __builtin_amdgcn_make_buffer_rsrc(xn, (short)0, (int)((long)(a.H + a.T) * 32 * 4), BUF_DW3);
        float* nrow = nxt + r * XS;
        const bool halo_row = r >= TP - min(1 << ((l + 1) % a.nbl), TP);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          *(floatx4*)(nrow + 16 * rb + 4 * g) = accr[rb];
          const int off = ((a.H + t) * 32 + 16 * rb + 4 * g) * 4;
          if (valid && halo_row) __builtin_amdgcn_raw_buffer_store_b128(accr[rb], rn, off, 0, 16);
          if (valid && !halo_row) __builtin_amdgcn_raw_buffer_store_b128(accr[rb], rn, off, 0, 0);
        }
        FSTAMP(8);
        // the next layer's own tap from the row this wave's lanes just wrote (wave-local)
        wave_lds_fence();
        const float* Wn = img(l + 1);
        conv16_init(bias_of(Wn), cv, q0, h, acc);
        if (has_cond && l + 2 < a.L) load_cond16<CM>(a, l + 2, myid, m, valid, q0, h, cv);
        conv16_tap<LC ? 2 : 1>(nrow, (const unsigned short*)Wn + 96, i16, g, acc);
        if (LC && !LCLATE) lc16_terms(LCIu, lcv, i16, g, acc);
      }
      FSTAMP(5);
      // publish x_{l+1}: every wave drains its stores, barrier, one lane signals
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      FSTAMP(9);
      __syncthreads();
      FSTAMP(10);
      if (tid == 0 && l + 1 < a.L) publish_flag(a.flags + tile, (unsigned)(l + 1));
      if (LC && !LCLATE && l + 2 < a.L) dma_lc16_image<NW>(a.lcimg, l + 2, LCI, w, lane);
      if (DMAIMG && l + 2 < a.L) {
        const float* src = wsrc + (long)(l + 2) * IMGF + lane * 4;
        float* dst = IMG0 + (l & 1) * IMGF;
#pragma unroll
        for (int i = 0; i < IMGF / 256 / NW; ++i) dma16(src + (w + NW * i) * 256, dst + (w + NW * i) * 256);
      }
      // (LCLATE) the LC image of layer l+1 landed by the drain before the barrier above
      if (LCLATE && l + 1 < a.L) lc16_terms(LCIu, lcv, i16, g, acc);
      if (!DMAIMG && l + 2 < a.L) {
        float* dst = IMG0 + (l & 1) * IMGF;
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const int e = tid + NT * i;
          if (e < IMGF / 4) *(floatx4*)(dst + 4 * e) = pf[i];
        }
      }
      FSTAMP(6);
      if (!LC) store_zs();
      FSTAMP(7);
    }
#undef FSTAMP
  }
}

// ---- deferred slab reduction -------------------------------------------------------------

// Destination of slab column c (padded 32-channel layout) in reference layout.
LBWN_DEV void slab_store(const RedK& a, int c, float tot) {
  const int Cr = a.Cr, Cd = a.Cd;
  if (c < 4096) {
    const int cc = c & 2047, tap = cc >> 10, in = (cc >> 5) & 31, o = cc & 31;
    float* dst = c < 2048 ? a.dsig : a.dgate;
    if (in < Cr && o < Cd) dst[(tap * Cr + in) * Cd + o] = tot;
  } else if (c < 5120) {
    const int cc = c - 4096, zc = cc >> 5, o = cc & 31;
    if (zc < Cd && o < Cr) a.dres[zc * Cr + o] = tot;
  } else {
    const int cc = c - 5120, seg = cc >> 5, o = cc & 31;
    if (seg == 0 && a.dbsig && o < Cd) a.dbsig[o] = tot;
    if (seg == 1 && a.dbgate && o < Cd) a.dbgate[o] = tot;
    if (seg == 2 && a.dbres && o < Cr) a.dbres[o] = tot;
  }
}

// Column group `grp` (32 columns) summed over all parts: thread = (part lane p8, column);
// `pre` holds parts p8, p8+8, ... (up to RED_PARTS) loaded earlier.
LBWN_DEV void slab_group_finish(const RedK& a, int grp, const float (&pre)[RED_PARTS], float* scratch,
                                int tid) {
  const int c = grp * 32 + (tid & 31), p8 = tid >> 5;
  float s = 0.f;
  if (c < SLAB) {
#pragma unroll
    for (int j = 0; j < RED_PARTS; ++j) s += pre[j];
    for (int p = p8 + 8 * RED_PARTS; p < a.nparts; p += 8) s += a.slab[(long)p * a.stride + c];
  }
  scratch[tid] = s;
  __syncthreads();
  if (tid < 32 && c < SLAB) {
    float tot = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) tot += scratch[j * 32 + tid];
    slab_store(a, c, tot);
  }
  __syncthreads();
}

LBWN_DEV void slab_group_prefetch(const RedK& a, int grp, float (&pre)[RED_PARTS], int tid) {
  const int c = grp * 32 + (tid & 31), p8 = tid >> 5;
#pragma unroll
  for (int j = 0; j < RED_PARTS; ++j) {
    const int p = p8 + 8 * j;
    pre[j] = (c < SLAB && p < a.nparts) ? a.slab[(long)p * a.stride + c] : 0.f;
  }
}

// ---- persistent backward chain -------------------------------------------------------------
// Layers L-1 .. 0 in one launch; tiles in DECREASING order (layer l's tile needs dx_{l+1} at
// rows t + d_{l+1}, i.e. from the same or LATER tiles).  dx_{l+1}[t] = out_a[t] + out_c0[t+d']
// (tmodel.py:122-127 autodiff): out_a never leaves the block (registers, acc layout = the B
// operand of the next dz product); out_c0 stays in LDS for the block's own rows and only its
// first min(d,128) rows are published (sc1) to the per-layer hand-off buffer for the tile
// below.  The gate recompute runs before the hand-off wait and the weight-gradient products
// after the publish, so the cross-tile critical path per layer is G-build → dz → dx.
// Weight-gradient partials go to slab[l][tile] (summed by layer_reduce_all_kernel).
struct ChainBK {
  int xcd;                     // chain_first: XCD-grouped tile walk
  const float* X; long xls;
  const float* DZ; long lddz; long dzls;   // dzls > 0: DZ in chain order (sg_off blocks per layer)
  const float* wpack;
  float* slab;                 // [L][ntiles][SLAB]
  float* ocg; long ocls;       // out_c0 hand-off rows: [L][B·T][32], layer stride ocls floats
  float* dx0_a; float* dx0_c;  // layer 0's out_a / out_c0 [B·T][32]
  const float* gc_tab; long gc_ld; const int* ids; const float* cond; long ldcond;
  float* dv_out; long lddv;    // dv export for the LC gradients: [M][L·2Cd] (layer l at column l·2Cd) or null
  long dvks;                   // x3 forms: 0, or the chunk stride of the k-blocked export [L·2][Mp][32]
  float* gc_dtab;              // GC gradient table, layout of gc_tab, atomics, or null
  unsigned* flags; unsigned* status;
  int B, T, H, L, nbl, Cd;
  long long* trace; int trace_blk;   // debug stamps (null in production)
  // bf16-split form (chain_bwd_x3_kernel): z rows (row stride lddz), σ rows [L][M][32], images
  const float* Zf; const float* SG; long sgls; const float* bimg;
  int* tile_gid;               // GC: per tile its uniform voice id or -1 (x3 chain), or null
  float* gx; long gxls;        // chain_bwd16_kernel<.., false>: G export [L][Mp][32] (layer stride gxls)
};

// dv rows of wave w's 32 positions (DV, position-major) scatter-added into the GC gradient
// table row (row stride ld) of each position's voice id.  uni_id >= 0: the caller knows the
// run is one id (one atomic per column); otherwise the ids are checked here.
LBWN_DEV void gc_scatter(float* gtab, long ld, const int* ids_b, const float* DV, int t0, int T, int w, int lane,
                         int Cd, int uni_id) {
  const int tw0 = t0 + 32 * w;
  const int nv = min(32, T - tw0);
  if (nv <= 0) return;
  const int* idw = ids_b + tw0;
  int id0 = uni_id;
  if (id0 < 0) {
    id0 = idw[0];
    bool uni = true;
    for (int p = 1; p < nv; ++p) uni &= (idw[p] == id0);
    if (!uni) id0 = -1;
  }
  const int o = lane, oc = o & 31;
  const float* dvw = DV + 32 * w * DS;
  if (oc >= Cd) return;
  const int col = o < 32 ? oc : Cd + oc;
  if (id0 >= 0) {
    float s = 0.f;
    for (int p = 0; p < nv; ++p) s += dvw[p * DS + o];
    atomicAdd(gtab + (long)id0 * ld + col, s);
  } else {   // one atomic per run of equal ids (as gc_scatter_x3)
    int p = 0;
    while (p < nv) {
      const int id = idw[p];
      float s = 0.f;
      for (; p < nv && idw[p] == id; ++p) s += dvw[p * DS + o];
      atomicAdd(gtab + (long)id * ld + col, s);
    }
  }
}

// Xp Xc | IMG | DV | G | OC | XpN XcN (the next layer's rows, DMA-staged, unpadded): 163,712 B
constexpr int CB_LDS = 2 * LP * XS + WIMG + LP * DS + 2 * LP * XS + 2 * LP * 32;
static_assert(CB_LDS * 4 + 16 <= 160 * 1024, "chain bwd LDS");

// next-layer rows by LDS-DMA: wave w moves rows [32w, 32w+32) of the dilated-tap and own-row
// blocks, 8 rows (1 KiB) per global_load_lds_dwordx4; rows past T are clamped here and zeroed
// by the copy
LBWN_DEV void dma_rows(float* XpN, float* XcN, const float* xl, int t0, int d, int T, int H, int w, int lane,
                       int j0, int j1) {
#pragma unroll
  for (int j = j0; j < j1; ++j) {
    const int row = 32 * w + 8 * j + (lane >> 3), c4 = (lane & 7) * 4;
    const int trow = min(t0 + row, T - 1);
    __builtin_amdgcn_global_load_lds(xl + (long)(H + trow - d) * 32 + c4,
                                     (__attribute__((address_space(3))) void*)(XpN + (32 * w + 8 * j) * 32), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(xl + (long)(H + trow) * 32 + c4,
                                     (__attribute__((address_space(3))) void*)(XcN + (32 * w + 8 * j) * 32), 16, 0, 0);
  }
}
// unpadded staged rows -> padded tile rows (zero past T)
LBWN_DEV void copy_rows(float* dst, const float* src, int t0, int T, int tid) {
  floatx4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    v[i] = *(const floatx4*)(src + (e >> 3) * 32 + (e & 7) * 4);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    if (t0 + (e >> 3) >= T) v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    *(floatx4*)(dst + (e >> 3) * XS + (e & 7) * 4) = v[i];
  }
}

__global__ __launch_bounds__(256) void chain_bwd_kernel(ChainBK a) {
  __shared__ __attribute__((aligned(16))) float sm[CB_LDS];
  __shared__ int s_fail;
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* Ws = Xc + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* DV = Ws + WIMG;
  float* G = DV + LP * DS;
  float* OC = G + LP * XS;
  float* XpN = OC + LP * XS;    // next layer's rows, DMA-staged during this layer
  float* XcN = XpN + LP * 32;
  float* ZT = Ws;   // after dx
  float* RED = Xp;  // after dSIG
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int r = 32 * w + pi;
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;
  const int oc_bytes = (int)std::min<long>(a.ocls * 4, 0x7fffffffL);
  if (tid == 0) s_fail = 0;
  const int first = chain_first(a.xcd);
  for (int it = first; it < ntiles; it += gridDim.x) {
    const int tile = ntiles - 1 - it;
    const int b = tile / tps, tt = tile % tps, t0 = tt * LP;
    const int t = t0 + r;
    const bool valid = t < a.T;
    const long mb = (long)b * a.T, m = mb + t;
    const long sb = (long)b * (a.H + a.T) * 32;
    const bool has_cond = a.gc_tab || a.cond;
    const int myid = (a.gc_tab && valid) ? a.ids[m] : 0;
    floatx4 cv[8];
    load_cond<2>(a, a.L - 1, myid, m, valid && has_cond, h, cv);
    // GC grads: is this wave's 32-position run one voice id?  (fast scatter path)
    const int wave_id = __shfl(myid, 0);
    const bool wave_uni = __all(!valid || myid == wave_id);
    __syncthreads();
    stage_image(Ws, a.wpack + (long)(a.L - 1) * WIMG, tid);
    floatx16 oa;  // out_a of layer l+1, own row
#pragma unroll
    for (int q = 0; q < 16; ++q) oa[q] = 0.f;
    const bool trc = a.trace && (int)blockIdx.x == a.trace_blk && tid == 0 && it == first;
#define CSTAMP(i) if (trc) a.trace[16 * l + (i)] = clock64()
    for (int l = a.L - 1; l >= 0; --l) {
      CSTAMP(0);
      const int d = 1 << (l % a.nbl);
      const int dn = (l + 1 < a.L) ? 1 << ((l + 1) % a.nbl) : 0;
      const float* xl = a.X + (long)l * a.xls + sb;
      // 0. this layer's inputs: x_l taps / own rows (the tile's first layer: from HBM; later
      //    layers: DMA-staged during the previous layer, landed by its publish drain + barrier),
      //    dZ rows (first used after the gate recompute and G build); next image prefetch
      if (l == a.L - 1) {
        stage_rows(Xp, xl, t0, -d, a.T, a.H, 32, tid);
        stage_rows(Xc, xl, t0, 0, a.T, a.H, 32, tid);
      } else {
        copy_rows(Xp, XpN, t0, a.T, tid);
        copy_rows(Xc, XcN, t0, a.T, tid);
      }
      floatx16 dz;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 v = *(const floatx4*)(a.DZ + (mb + min(t, a.T - 1)) * a.lddz + (long)l * a.Cd + 8 * q + 4 * h);
        if (!valid) v = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) dz[4 * q + j] = v[j];
      }
      floatx4 pf[IMG_PF];
      if (l > 0) {
        const floatx4* src = (const floatx4*)(a.wpack + (long)(l - 1) * WIMG);
#pragma unroll
        for (int i = 0; i < IMG_PF; ++i) {
          const int e = tid + 256 * i;
          pf[i] = src[min(e, WIMG / 4 - 1)];   // clamped: no load behind a branch
        }
      }
      __syncthreads();
      CSTAMP(1);
      // the next layer's rows into XpN / XcN (everyone has copied them out: the barrier above),
      // half before each conv half so the DMA issue overlaps in-flight MFMAs
      const float* xnext = a.X + (long)(l > 0 ? l - 1 : 0) * a.xls + sb;
      const int dnext = 1 << ((l > 0 ? l - 1 : 0) % a.nbl);
      if (l > 0) dma_rows(XpN, XcN, xnext, t0, dnext, a.T, a.H, w, lane, 0, 2);
      // 1. recompute the gate (no cross-tile dependency)
      floatx16 acc_s, acc_g;
      conv_init(bs, cv, h, acc_s, acc_g);
      if (has_cond && l > 0) load_cond<2>(a, l - 1, myid, m, valid, h, cv);
      conv_half(Xc + r * XS, Ws + 32 * WS, pi, h, acc_s, acc_g);
      if (l > 0) dma_rows(XpN, XcN, xnext, t0, dnext, a.T, a.H, w, lane, 2, 4);
      conv_half(Xp + r * XS, Ws, pi, h, acc_s, acc_g);
      floatx16 th, sg;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        th[q] = tanhf_(acc_s[q]);
        sg[q] = sigmoidf_(acc_g[q]);
      }
      CSTAMP(2);
      // 2. G = dx_{l+1} rows of this tile: out_c0_{l+1}[t + dn] (own LDS / published rows) + out_a
      if (dn) {
        const int ptt = tt + max(1, dn / LP);
        if (ptt < tps) {
          if (tid == 0 && !s_fail) {
            if (!wait_flag_ge(a.flags + (long)b * tps + ptt, (unsigned)(a.L - l - 1), a.status, 2u)) s_fail = 1;
          }
          __syncthreads();
        }
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)(l + 1) * a.ocls, (short)0, oc_bytes, BUF_DW3);
        // rows from the own tile's OC (LDS) or the producer's published rows (sc1 loads): all
        // loads issued unconditionally at clamped indices, then selected (no load behind a branch)
        floatx4 gl[4], go[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = tid + 256 * i, row = e >> 3, c4 = (e & 7) * 4, sr = row + dn;
          const int ts = min(t0 + sr, a.T - 1);
          gl[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((mb + ts) * 32 + c4) * 4), 0, 16);
          go[i] = *(const floatx4*)(OC + min(sr, LP - 1) * XS + c4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = tid + 256 * i, row = e >> 3, c4 = (e & 7) * 4, sr = row + dn, ts = t0 + sr;
          floatx4 v = sr < LP ? go[i] : gl[i];
          if (ts >= a.T) v = floatx4{0.f, 0.f, 0.f, 0.f};
          *(floatx4*)(G + row * XS + c4) = v;
        }
        __syncthreads();
      }
      CSTAMP(3);
      floatx16 gv;
      {  // own row: + out_a (at the top layer g = 0: the row is written here, not read)
        float* grow = G + r * XS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          floatx4 v = dn ? *(const floatx4*)(grow + 8 * q + 4 * h) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] += oa[4 * q + j]; gv[4 * q + j] = v[j]; }
          *(floatx4*)(grow + 8 * q + 4 * h) = v;
        }
      }
      // 3. dz += RES·g; dv
      {
        floatx4 rx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rx[q] = *(const floatx4*)(Rs + pi * XS + 8 * q + 4 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) dz = mfma32(rx[q][j], gv[4 * q + j], dz);
      }
      floatx16 dvs, dvg;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        dvs[q] = dz[q] * sg[q] * (1.f - th[q] * th[q]);
        dvg[q] = dz[q] * th[q] * sg[q] * (1.f - sg[q]);
      }
      {
        float* dvrow = DV + r * DS;
        float* dvo = (a.dv_out && valid) ? a.dv_out + m * a.lddv + (long)l * 64 : nullptr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 vs = floatx4{dvs[4 * q], dvs[4 * q + 1], dvs[4 * q + 2], dvs[4 * q + 3]};
          const floatx4 vg = floatx4{dvg[4 * q], dvg[4 * q + 1], dvg[4 * q + 2], dvg[4 * q + 3]};
          *(floatx4*)(dvrow + 8 * q + 4 * h) = vs;
          *(floatx4*)(dvrow + 32 + 8 * q + 4 * h) = vg;
          if (dvo) {
            *(floatx4*)(dvo + 8 * q + 4 * h) = vs;
            *(floatx4*)(dvo + 32 + 8 * q + 4 * h) = vg;
          }
        }
      }
      CSTAMP(4);
      // 4. dx: out_a = g + W1·dv, out_c0 = W0·dv
      floatx16 acc_a = gv, acc_c;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc_c[q] = 0.f;
      {
        floatx4 wv[2][4];
        auto loadw = [&](int q, int buf) {
          const int ko = 8 * q + 4 * h;
          wv[buf][0] = *(const floatx4*)(Ws + pi * WS + ko);
          wv[buf][1] = *(const floatx4*)(Ws + pi * WS + 32 + ko);
          wv[buf][2] = *(const floatx4*)(Ws + (32 + pi) * WS + ko);
          wv[buf][3] = *(const floatx4*)(Ws + (32 + pi) * WS + 32 + ko);
        };
        loadw(0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cb = q & 1;
          if (q + 1 < 4) loadw(q + 1, cb ^ 1);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int s2 = 4 * q + j;
            acc_a = mfma32(wv[cb][2][j], dvs[s2], acc_a);
            acc_c = mfma32(wv[cb][0][j], dvs[s2], acc_c);
            acc_a = mfma32(wv[cb][3][j], dvg[s2], acc_a);
            acc_c = mfma32(wv[cb][1][j], dvg[s2], acc_c);
          }
        }
      }
      {
        float* ocrow = OC + r * XS;
        const __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)l * a.ocls, (short)0, oc_bytes, BUF_DW3);
        const bool pub = l > 0 && valid && r < min(d, LP);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 v = floatx4{acc_c[4 * q], acc_c[4 * q + 1], acc_c[4 * q + 2], acc_c[4 * q + 3]};
          *(floatx4*)(ocrow + 8 * q + 4 * h) = v;
          if (pub) __builtin_amdgcn_raw_buffer_store_b128(v, rw, (int)((m * 32 + 8 * q + 4 * h) * 4), 0, 16);
        }
      }
      if (l == 0 && valid) {
        store_rows16(a.dx0_a + m * 32, acc_a, 32, h);
        store_rows16(a.dx0_c + m * 32, acc_c, 32, h);
      }
      oa = acc_a;
      CSTAMP(5);
      // publish out_c0_l (every wave drains its sc1 stores, barrier, one lane signals)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // also: DV complete, the weight image is dead
      if (tid == 0 && l > 0) publish_flag(a.flags + tile, (unsigned)(a.L - l));
      if (a.gc_dtab) gc_scatter(a.gc_dtab + (long)l * 64, a.gc_ld, a.ids + mb, DV, t0, a.T, w, lane, 32,
                                wave_uni ? wave_id : -1);
      CSTAMP(6);
      // 5. weight gradients of layer l over this tile
      {
        float* zrow = ZT + r * XS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          floatx4 zv;
#pragma unroll
          for (int j = 0; j < 4; ++j) zv[j] = th[4 * q + j] * sg[4 * q + j];
          *(floatx4*)(zrow + 8 * q + 4 * h) = zv;
        }
      }
      floatx16 accW, accR;
#pragma unroll
      for (int q = 0; q < 16; ++q) { accW[q] = 0.f; accR[q] = 0.f; }
      {  // dSIG/dGATE tile w: A[i=in][k=pos] = X[pos][in], B[k][j=o] = DV[pos][o]
        // Operands for 16 MFMAs are read one chunk ahead; the sched_barriers keep hipcc from
        // sinking each read next to its MFMA (at this kernel's register pressure it otherwise
        // does, and every MFMA waits out an LDS round trip: ~3.5x the MFMA time)
        const float* X = (w & 1) ? Xc : Xp;
        const int oc = (w >> 1) * 32 + pi;
        float xa[2][16], da[2][16];
        auto loadc = [&](int c, int buf) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int p = 2 * (16 * c + i) + h;
            xa[buf][i] = X[p * XS + pi];
            da[buf][i] = DV[p * DS + oc];
          }
        };
        loadc(0, 0);
#pragma unroll
        for (int c = 0; c < LP / 32; ++c) {
          const int cb = c & 1;
          if (c + 1 < LP / 32) loadc(c + 1, cb ^ 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 16; ++i) accW = mfma32(xa[cb][i], da[cb][i], accW);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      CSTAMP(7);
      __syncthreads();  // ZT visible; Xp/Xc free for RED
      {  // dRES part over this wave's 32 positions (all operands read before the first MFMA)
        float za[16], ga[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const int p = 32 * w + 2 * s2 + h;
          za[s2] = ZT[p * XS + pi];
          ga[s2] = G[p * XS + pi];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) accR = mfma32(za[s2], ga[s2], accR);
      }
      CSTAMP(8);
      float* slab = a.slab + ((long)l * ntiles + tile) * SLAB;
      {  // bias partials: column sums of DV (64) and G (32)
        float* part = RED + 4096;  // [8][96] after the dRES exchange area
        if (tid < 128) {
          const int c4 = (tid & 15) * 4, pc = tid >> 4;
          floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int p = 0; p < 16; ++p) s4 += *(const floatx4*)(DV + (pc * 16 + p) * DS + c4);
          *(floatx4*)(part + pc * 96 + c4) = s4;
        } else if (tid < 192) {
          const int c4 = ((tid - 128) & 7) * 4, pc = (tid - 128) >> 3;
          floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int p = 0; p < 16; ++p) s4 += *(const floatx4*)(G + (pc * 16 + p) * XS + c4);
          *(floatx4*)(part + pc * 96 + 64 + c4) = s4;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          slab[w * 1024 + acc_row(q, h) * 32 + pi] = accW[q];
          RED[w * 1024 + acc_row(q, h) * 32 + pi] = accR[q];
        }
        __syncthreads();
        if (tid < 96) {
          float s1 = 0.f;
#pragma unroll
          for (int pc = 0; pc < 8; ++pc) s1 += part[pc * 96 + tid];
          slab[5120 + tid] = s1;
        }
        for (int e = tid; e < 1024; e += 256)
          slab[4096 + e] = ((RED[e] + RED[1024 + e]) + RED[2048 + e]) + RED[3072 + e];
      }
      CSTAMP(9);
      // 6. next layer's weight image (ZT is dead: every wave passed the barrier after dRES)
      if (l > 0) {
#pragma unroll
        for (int i = 0; i < IMG_PF; ++i) {
          const int e = tid + 256 * i;
          if (e < WIMG / 4) *(floatx4*)(Ws + 4 * e) = pf[i];
        }
      }
      __syncthreads();
      CSTAMP(10);
    }
#undef CSTAMP
  }
}

// ---- backward chain on the bf16 cores (the X3 arithmetic of DESIGN §4.0) -----------------------
// Same tile walk, hand-off and slab layout as chain_bwd_kernel; what changes:
//  * no gate recompute: the X3 forward chain stores σ(v_gate) (SG [L][M][32]) beside z (Zcat),
//    so tanh = z·σ⁻¹ and dv come from two row loads (prefetched a layer ahead) instead of a
//    second 64-channel conv;
//  * dx = W·dv (K = 64) and the weight gradients dSIG/dGATE = Xᵀ·DV (K = 128 positions) and
//    dRES = Zᵀ·G run on v_mfma_f32_32x32x16_bf16 / 16x16x32 from exact 3-term splits (six
//    products); dz = dZ + RES·g (16 f32 MFMAs) stays on v_mfma_f32_32x32x2_f32;
//  * this layer's x rows (both taps) and z rows are LDS-DMA'd into unpadded tiles during the
//    G build, the next layer's weight image right after the publish; DV, G and OC live in
//    32-float rows with an XOR swizzle of the 4-float groups (swz) so that both the own-row
//    b128 writes and the column reads of the weight-gradient products are conflict-free.
// Backward image per layer: WD[tap][in][plane][kk] (bf16, row XW_ROW) with kk = 16s+8h+j holding
// out channel o = 32(s>>1) + 16(s&1) + 8(j>>2) + 4h + (j&3) (sig 0..31 | gate 32..63): the k order
// of the dv registers used as the B operand; then Rs f32 [c][XS] for the dz product of
// chain_bwd_x3_kernel, padded to a whole number of 1-KiB DMA pieces (BX_F: what that kernel
// loads); then RX, the same residual weights split for chain_bwd16_kernel's dz on the bf16 cores:
// RX[c][plane][kk] (bf16, row RX_ROW) with kk = 8g + e holding res channel 16(e >> 2) + 4g + (e & 3)
// (the order of the lane's two N-layout g registers).  chain_bwd16_kernel loads WD and RX only
// (B16IMG_F floats: global pieces [0, BD_PC) and [RX_GPC, RX_GPC + RX_PC)).
constexpr int BD_US = 2 * 32 * XW_ROW;
constexpr int BX_F = (BD_US / 2 + 32 * XS + 255) / 256 * 256;   // 7680 floats
// 224-B RX rows (14 16-B slots): the 16x16x32 A-fragment reads (rows ch16(bb, i), slot 4p + g) hit
// 16 distinct slots in every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS)
constexpr int RX_ROW = 112;
constexpr int RX_F = 32 * RX_ROW / 2;                          // 1792 floats
constexpr int BIMG_F = BX_F + RX_F;                            // 9472 floats: global stride per layer
constexpr int B16IMG_F = BD_US / 2 + RX_F;                     // 8192 floats in chain_bwd16_kernel's LDS
constexpr int BD_PC = BD_US / 2 / 256, RX_GPC = BX_F / 256, RX_PC = RX_F / 256;
static_assert(BD_US / 2 % 256 == 0 && RX_F % 256 == 0 && B16IMG_F % 256 == 0, "bwd image: whole DMA pieces");
constexpr int CBX_LDS = BX_F + 7 * LP * 32 + 8 * 96;              // IMG | Xp Xc ZT | DVs DVg G OC | part
static_assert(CBX_LDS * 4 + 16 <= 160 * 1024, "chain bwd x3 LDS");

LBWN_DEV void pack_bx3_body(int l, const float* sig, const float* gate, const float* res, float* out, int Cr, int Cd) {
  const float* ws = sig + (long)l * 2 * Cr * Cd;
  const float* wg = gate + (long)l * 2 * Cr * Cd;
  const float* wr = res + (long)l * Cd * Cr;
  float* img = out + (long)l * BIMG_F;
  unsigned short* wd = (unsigned short*)img;
  for (int e = threadIdx.x; e < 2 * 32 * 32; e += blockDim.x) {
    const int tap = e >> 10, in = (e >> 5) & 31, kk = 2 * (e & 31);
    floatx2 x = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k2 = kk + u, s2 = k2 >> 4, hh = (k2 >> 3) & 1, j = k2 & 7;
      const int o = 32 * (s2 >> 1) + 16 * (s2 & 1) + 8 * (j >> 2) + 4 * hh + (j & 3), oc = o & 31;
      const float* wk = o < 32 ? ws : wg;
      if (in < Cr && oc < Cd) x[u] = wk[(tap * Cr + in) * Cd + oc];
    }
    unsigned hi, mi, lo;
    split2(x, hi, mi, lo);
    unsigned short* row = wd + (tap * 32 + in) * XW_ROW + kk;
    *(unsigned*)(row) = hi;
    *(unsigned*)(row + 64) = mi;
    *(unsigned*)(row + 128) = lo;
  }
  float* rs = img + BD_US / 2;
  for (int e = threadIdx.x; e < 32 * XS; e += blockDim.x) {
    const int c = e / XS, o = e % XS;
    rs[e] = (c < Cd && o < Cr) ? wr[c * Cr + o] : 0.f;
  }
  for (int e = BD_US / 2 + 32 * XS + threadIdx.x; e < BX_F; e += blockDim.x) img[e] = 0.f;
  unsigned short* rx = (unsigned short*)(img + BX_F);
  for (int e = threadIdx.x; e < 32 * 16; e += blockDim.x) {
    const int c = e >> 4, kk = 2 * (e & 15);
    floatx2 x = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k2 = kk + u, gg = k2 >> 3, ee = k2 & 7, o = 16 * (ee >> 2) + 4 * gg + (ee & 3);
      if (c < Cd && o < Cr) x[u] = wr[c * Cr + o];
    }
    unsigned hi, mi, lo;
    split2(x, hi, mi, lo);
    unsigned short* row = rx + c * RX_ROW + kk;
    *(unsigned*)(row) = hi;
    *(unsigned*)(row + 32) = mi;
    *(unsigned*)(row + 64) = lo;
  }
}

__global__ void pack_layers_x3_kernel(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                      const float* res, const float* res_b, unsigned short* out, int Cr, int Cd) {
  pack_x3_body(blockIdx.x, sig, gate, sig_b, gate_b, res, res_b, out, Cr, Cd);
}
__global__ void pack_layers_bx3_kernel(const float* sig, const float* gate, const float* res, float* out, int Cr,
                                       int Cd) {
  pack_bx3_body(blockIdx.x, sig, gate, res, out, Cr, Cd);
}
// both chains' images in one launch (blocks [0, L): forward, [L, 2L): backward), and in the
// blocks after them (if skip_b) the skip GEMM's bias Σ_l skip_b[l] (l in order)
LBWN_DEV void pack_fb_x3_block(int l, const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                               const float* res, const float* res_b, unsigned short* fout, float* bout, int L, int Cr,
                               int Cd, const float* skip_b, int Cs, float* bsum, const float* lc_sig,
                               const float* lc_gate, int Lo, unsigned short* lcout, int lc16) {
  const int nlc = lcout ? L : 0;
  if (l < L) {
    pack_x3_body(l, sig, gate, sig_b, gate_b, res, res_b, fout, Cr, Cd);
  } else if (l < 2 * L) {
    pack_bx3_body(l - L, sig, gate, res, bout, Cr, Cd);
  } else if (l < 2 * L + nlc) {
    if (lc16) pack_lc16_body(l - 2 * L, lc_sig, lc_gate, lcout, Lo, Cd);
    else pack_lc_x3_body(l - 2 * L, lc_sig, lc_gate, lcout, Lo, Cd);
  } else {
    const int n = (l - 2 * L - nlc) * 256 + threadIdx.x;
    if (n < Cs) {
      float s = 0.f;
#pragma unroll 10
      for (int k = 0; k < L; ++k) s += skip_b[(long)k * Cs + n];
      bsum[n] = s;
    }
  }
}
__global__ __launch_bounds__(256) void pack_layers_fb_x3_kernel(const float* sig, const float* gate,
                                                                const float* sig_b, const float* gate_b,
                                                                const float* res, const float* res_b,
                                                                unsigned short* fout, float* bout, int L, int Cr,
                                                                int Cd, const float* skip_b, int Cs, float* bsum,
                                                                const float* lc_sig, const float* lc_gate, int Lo,
                                                                unsigned short* lcout, int lc16) {
  pack_fb_x3_block(blockIdx.x, sig, gate, sig_b, gate_b, res, res_b, fout, bout, L, Cr, Cd, skip_b, Cs, bsum, lc_sig,
                   lc_gate, Lo, lcout, lc16);
}

// The step's start-of-step work in ONE launch (lbwn_step_prologue_launch): zero the status word and
// hand-off flags, pre-split the skip/head weight planes, gather the PRE embedding, prepend the
// D-sep state, and pack both chains' images -- five independent jobs that ran as five dependent
// launches of 7-12 us each (profiles/r04_v1_step_timeline.txt).  Block ranges, heavy jobs first.
struct PrologueK {
  lbwn_prologue_args a;
  SplitJobs jb;
  int nz, ns, ne, nd, np;   // blocks: zero, split (per job), embed, D-sep (all layers), pack
  bool ev4, dv4;            // float4 items: embed, D-sep
};
__global__ __launch_bounds__(256) void step_prologue_kernel(PrologueK k) {
  const lbwn_prologue_args& a = k.a;
  long b = blockIdx.x;
  if (b < (long)k.ns * a.njobs) {
    split_planes_body(k.jb, (int)(b / k.ns), b % k.ns, k.ns);
    return;
  }
  b -= (long)k.ns * a.njobs;
  if (b < k.ne) {
    embed_flat_body(b, k.ne, a.q, a.pre, a.pre_b, a.X, a.B, a.T, a.H, a.Cr, a.Q, k.ev4);
    return;
  }
  b -= k.ne;
  if (b < k.nd) {
    dsep_flat_body<true>(b, k.nd, a.X, a.xls, const_cast<float*>(a.save), a.L, a.nbl, a.B, a.T, a.H, a.Cr, k.dv4);
    return;
  }
  b -= k.nd;
  if (b < k.nz) {
    zero_body(b, k.nz, (unsigned*)a.zero, (long)(a.zero_bytes / 4));
    return;
  }
  b -= k.nz;
  pack_fb_x3_block((int)b, a.sig, a.gate, a.sig_b, a.gate_b, a.res, a.res_b, a.fout, a.bout, a.L, a.Cr, a.Cd,
                   a.skip_b, a.Cs, a.bsum, a.lc_sig, a.lc_gate, a.Lo, a.lcout, a.lc16);
}

// element (p, c) of a 32-float-row tile with the 4-float groups XOR-permuted: bit 4 of the column
// by row parity, bits 2-3 by (p >> 1) & 3.  Eight consecutive rows (the 8 lanes of one
// ds_write_b128 group writing the same column group of their own rows) land on 8 distinct groups:
// conflict-free; rows p, p+1 read by the two lane halves of a b32 read fall in opposite 16-bank
// halves (a row-pair permutation left those writes 2-way conflicted: 6.6M of the kernel's 15.6M
// SQ_LDS_BANK_CONFLICT cycles, tools/lds_conf.sh)
LBWN_DEV int swz(int p, int c) { return p * 32 + (c ^ (((p & 1) << 4) | (((p >> 1) & 3) << 2))); }

// acc += A·B over one 32-deep k-step of v_mfma_f32_16x16x32_bf16 from split fragments
LBWN_DEV floatx4 mfma16_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// GC rows of a wave whose 32 positions are not one voice: dv column sums per run of equal ids
// (ids change only at file boundaries), one atomic per run and column.  The runs come from the
// lanes' own ids (lane p of either half holds position 32w + p; -1 past the end): run starts =
// ballot of id changes, computed once per tile by the caller (`starts`, bit p = a run starts at
// position p; `pid` = the lane's id).  No global loads: the old per-position loop loaded each id
// inside the loop and waited on every one (arch5 backward chain 550 -> 900 us on such batches).
LBWN_DEV void gc_scatter_x3(float* gtab, long ld, const float* DVs, const float* DVg, int w, int lane, int Cd,
                            unsigned starts, int pid) {
  const int o = lane, oc = o & 31;
  const float* pl = o < 32 ? DVs : DVg;
  const int col = o < 32 ? oc : Cd + oc;
  unsigned rest = starts;
  while (rest) {   // wave-uniform
    const int p0 = __ffs(rest) - 1;
    rest &= rest - 1;
    const int p1 = rest ? __ffs(rest) - 1 : 32;
    const int id = __shfl(pid, p0);
    if (id < 0) continue;   // positions past T
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += pl[swz(32 * w + p, oc)];
    if (oc < Cd) atomicAdd(gtab + (long)id * ld + col, s);
  }
}

template <bool TR>
__global__ __launch_bounds__(256) void chain_bwd_x3_kernel(ChainBK a) {
  __shared__ __attribute__((aligned(16))) float sm[CBX_LDS];
  __shared__ int s_fail;
  float* IMG = sm;
  const unsigned short* WD = (const unsigned short*)IMG;
  const float* Rs = IMG + BD_US / 2;
  float* Xp = IMG + BX_F;
  float* Xc = Xp + LP * 32;
  float* ZT = Xc + LP * 32;
  float* DVs = ZT + LP * 32;
  float* DVg = DVs + LP * 32;
  float* G = DVg + LP * 32;
  float* OC = G + LP * 32;
  float* part = OC + LP * 32;   // [8][96] bias partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int r = 32 * w + pi;
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;
  const int oc_bytes = (int)std::min<long>(a.ocls * 4, 0x7fffffffL);
  if (tid == 0) s_fail = 0;
  const int first = chain_first(a.xcd);
  for (int it = first; it < ntiles; it += gridDim.x) {
    const int tile = ntiles - 1 - it;
    const int b = tile / tps, tt = tile % tps, t0 = tt * LP;
    const int t = t0 + r;
    const bool valid = t < a.T;
    const long mb = (long)b * a.T, m = mb + t, mc = mb + min(t, a.T - 1);
    const long sb = (long)b * (a.H + a.T) * 32;
    const int myid = (a.gc_tab && valid) ? a.ids[m] : 0;
    const int wave_id = __shfl(myid, 0);
    const bool wave_uni = __all(!valid || myid == wave_id);
    // GC grads: a tile whose valid positions share one voice id (the common case: ids change only
    // at file boundaries) contributes its dv column sums -- the bias partials in its slab, computed
    // anyway -- to that id's row; lbwn_gc_tile_sum_launch adds them after the chain in tile order
    // (tile_gid[tile] = the id, or -1: this chain scatters the tile's rows itself).  64 atomics
    // per tile and layer onto the few voice rows serialised at L2 and stretched the publish drains.
    const int tile_id = a.gc_tab ? a.ids[mb + t0] : 0;
    const bool tile_uni = __syncthreads_and(!valid || myid == tile_id);
    if (a.tile_gid && tid == 0) a.tile_gid[tile] = tile_uni ? tile_id : -1;
    // this wave's id runs (gc_scatter_x3): lane pi's position id, -1 past T; bit p = a run starts at p
    const int gc_pid = valid ? myid : -1;
    const int gc_prev = __shfl(gc_pid, max(pi - 1, 0));
    const unsigned gc_starts = (unsigned)(__ballot(h == 0 && (pi == 0 || gc_pid != gc_prev)) & 0xffffffffull);
    // per-layer rows of this lane's position: dZ, z, σ (issued a layer ahead)
    floatx4 dzr[4], zr[4], sgr[4];
    auto load_regs = [&](int l) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dzr[q] = *(const floatx4*)(a.DZ + l * a.dzls + sg_off(mc, q, h));   // chain order: 1-KiB runs
        zr[q] = *(const floatx4*)(a.Zf + mc * a.lddz + (long)l * 32 + 8 * q + 4 * h);
        sgr[q] = *(const floatx4*)(a.SG + (long)l * a.sgls + sg_off(mc, q, h));
      }
    };
    auto dma_image = [&](int l) {
      const float* src = a.bimg + (long)l * BIMG_F + lane * 4;
      for (int i = w; i < BX_F / 256; i += 4) dma16(src + i * 256, IMG + i * 256);
    };
    __syncthreads();  // previous tile's LDS use done
    dma_image(a.L - 1);
    load_regs(a.L - 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    floatx16 oa;  // out_a of layer l+1, own row
#pragma unroll
    for (int q = 0; q < 16; ++q) oa[q] = 0.f;
    const bool trc = a.trace && (int)blockIdx.x == a.trace_blk && tid == 0 && it == first;
#define XSTAMP(i) if (TR && trc) a.trace[16 * l + (i)] = clock64()
    for (int l = a.L - 1; l >= 0; --l) {
      XSTAMP(0);
      const int d = 1 << (l % a.nbl);
      const int dn = (l + 1 < a.L) ? 1 << ((l + 1) % a.nbl) : 0;
      // 1. G = dx_{l+1} rows: out_c0_{l+1}[t + dn] (own OC / the producer's published rows) + out_a
      floatx4 gl[4], go[4];
      if (dn) {
        const int ptt = tt + max(1, dn / LP);
        if (ptt < tps) {
          if (tid == 0 && !s_fail) {
            if (!wait_flag_ge(a.flags + (long)b * tps + ptt, (unsigned)(a.L - l - 1), a.status, 2u)) s_fail = 1;
          }
          __syncthreads();
        }
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)(l + 1) * a.ocls, (short)0, oc_bytes, BUF_DW3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = tid + 256 * i, row = e >> 3, c4 = (e & 7) * 4, sr = row + dn;
          const int ts = min(t0 + sr, a.T - 1);
          gl[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((mb + ts) * 32 + c4) * 4), 0, 16);
          go[i] = *(const floatx4*)(OC + (CONF(1) ? 0 : swz(min(sr, LP - 1), c4)));
        }
      }
      if (dn) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = tid + 256 * i, row = e >> 3, c4 = (e & 7) * 4, sr = row + dn, ts = t0 + sr;
          floatx4 v = sr < LP ? go[i] : gl[i];
          if (ts >= a.T) v = floatx4{0.f, 0.f, 0.f, 0.f};
          *(floatx4*)(G + (CONF(2048) ? 4 * (tid & 255) : swz(row, c4))) = v;
        }
        // lands this wave's part of the weight image (LDS-DMA'd after the last layer's publish)
        // and the prefetched rows; the barrier then covers every wave's part
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      // the prefetched rows are consumed here, in the compiler's view, so that it has no load of
      // its own outstanding behind the DMA pieces below (its waits would count them)
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("" ::"v"(dzr[q]), "v"(zr[q]), "v"(sgr[q]));
      // this layer's x rows (x[t-d] | x[t]) and z rows by LDS-DMA into Xp / Xc / ZT (free since the
      // last layer's end barrier; first read after this layer's publish drain + barrier); the
      // pieces are issued between the dz MFMAs (row group j: 3 pieces)
      const float* xl = a.X + (long)l * a.xls + sb;
      auto dma_rows3 = [&](int j) {
        const int row = 32 * w + 8 * j + (lane >> 3), c4 = (lane & 7) * 4;
        const int trow = min(t0 + row, a.T - 1);
        if (CONF(1024)) return;
        dma16(xl + (long)(a.H + trow - d) * 32 + c4, Xp + (32 * w + 8 * j) * 32);
        dma16(xl + (long)(a.H + trow) * 32 + c4, Xc + (32 * w + 8 * j) * 32);
        dma16(a.Zf + (mb + trow) * a.lddz + (long)l * 32 + c4, ZT + (32 * w + 8 * j) * 32);
      };
      XSTAMP(1);
      floatx16 gv;
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // own row: + out_a (the top layer writes it, g = 0)
        float* gp = G + swz(r, 8 * q + 4 * h);
        floatx4 v = dn ? *(const floatx4*)(CONF(2) ? G : gp) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] += oa[4 * q + j]; gv[4 * q + j] = v[j]; }
        *(floatx4*)(CONF(2048) ? G + 4 * lane + 256 * q : gp) = v;
      }
      // 2. dz = dZ + RES·g  (f32 MFMA)
      floatx16 dz;
      {
        floatx4 rx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rx[q] = *(const floatx4*)(Rs + (CONF(4) ? 8 * q : pi * XS + 8 * q + 4 * h));
          floatx4 v = dzr[q];
          if (!valid) v = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) dz[4 * q + j] = v[j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int j = 0; j < 4; ++j) dz = mfma32(rx[q][j], gv[4 * q + j], dz);
          dma_rows3(q);
        }
      }
      // 3. dv from z and σ: tanh = z/σ (σ = 0 only where dv is 0 anyway)
      floatx16 dvs, dvg;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float zz = zr[q >> 2][q & 3], sg = sgr[q >> 2][q & 3];
        const float th = sg > 1e-30f ? zz * __builtin_amdgcn_rcpf(sg) : 0.f;
        dvs[q] = dz[q] * sg * (1.f - th * th);
        dvg[q] = dz[q] * zz * (1.f - sg);
      }
      {
        // DV export: rows (layer l at columns l·64) or k-blocked (a.dvks: [L·2][Mp][32] chunks)
        float* dvo = (a.dv_out && valid)
                         ? a.dv_out + (a.dvks ? 2L * l * a.dvks + m * 32 : m * a.lddv + (long)l * 64) : nullptr;
        const long dgo = a.dvks ? a.dvks : 32;   // gate half
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 vs = floatx4{dvs[4 * q], dvs[4 * q + 1], dvs[4 * q + 2], dvs[4 * q + 3]};
          const floatx4 vg = floatx4{dvg[4 * q], dvg[4 * q + 1], dvg[4 * q + 2], dvg[4 * q + 3]};
          *(floatx4*)(DVs + (CONF(2048) ? 4 * lane + 256 * q + 1024 * w : swz(r, 8 * q + 4 * h))) = vs;
          *(floatx4*)(DVg + (CONF(2048) ? 4 * lane + 256 * q + 1024 * w : swz(r, 8 * q + 4 * h))) = vg;
          if (dvo) {
            *(floatx4*)(dvo + 8 * q + 4 * h) = vs;
            *(floatx4*)(dvo + dgo + 8 * q + 4 * h) = vg;
          }
        }
      }
      XSTAMP(2);
      // 4. dx on the bf16 cores: out_a = g + W1·dv, out_c0 = W0·dv  (k-steps 0,1: sig; 2,3: gate)
      floatx16 acc_a = gv, acc_c;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc_c[q] = 0.f;
      {
        // fragments of k-step s+1 read while step s's MFMAs issue
        bf16x8 fa[2][3], fc[2][3];
        auto loadf = [&](int s2, int buf) {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            fa[buf][p] = *(const bf16x8*)(WD + (CONF(8) ? 64 * p + 16 * s2 : (32 + pi) * XW_ROW + 64 * p + 16 * s2 + 8 * h));
            fc[buf][p] = *(const bf16x8*)(WD + (CONF(8) ? 64 * p + 16 * s2 : pi * XW_ROW + 64 * p + 16 * s2 + 8 * h));
          }
        };
        loadf(0, 0);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int o8 = 8 * (s2 & 1), cb = s2 & 1;
          if (s2 + 1 < 4) loadf(s2 + 1, cb ^ 1);
          bf16x8 bx[3];
          if (s2 < 2)
            split8(floatx4{dvs[o8], dvs[o8 + 1], dvs[o8 + 2], dvs[o8 + 3]},
                   floatx4{dvs[o8 + 4], dvs[o8 + 5], dvs[o8 + 6], dvs[o8 + 7]}, bx);
          else
            split8(floatx4{dvg[o8], dvg[o8 + 1], dvg[o8 + 2], dvg[o8 + 3]},
                   floatx4{dvg[o8 + 4], dvg[o8 + 5], dvg[o8 + 6], dvg[o8 + 7]}, bx);
          acc_a = mfma_x3(fa[cb], bx, acc_a);
          acc_c = mfma_x3(fc[cb], bx, acc_c);
        }
      }
      {
        const __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)l * a.ocls, (short)0, oc_bytes, BUF_DW3);
        const bool pub = l > 0 && valid && r < min(d, LP);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 v = floatx4{acc_c[4 * q], acc_c[4 * q + 1], acc_c[4 * q + 2], acc_c[4 * q + 3]};
          *(floatx4*)(OC + (CONF(2048) ? 4 * lane + 256 * q + 1024 * w : swz(r, 8 * q + 4 * h))) = v;
          if (pub) __builtin_amdgcn_raw_buffer_store_b128(v, rw, (int)((m * 32 + 8 * q + 4 * h) * 4), 0, 16);
        }
      }
      if (l == 0 && valid) {
        store_rows16(a.dx0_a + m * 32, acc_a, 32, h);
        store_rows16(a.dx0_c + m * 32, acc_c, 32, h);
      }
      oa = acc_a;
      XSTAMP(3);
      // 5. publish out_c0_l (the drain also lands this layer's x / z DMA pieces)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // DV, G, Xp/Xc/ZT complete; the weight image is dead
      if (tid == 0 && l > 0) publish_flag(a.flags + tile, (unsigned)(a.L - l));
      // the next layer's weight image and rows are issued between the dSIG MFMAs below (landed
      // by the next layer's G build: vmcnt(0) + barrier)
      if (a.gc_dtab && !tile_uni) gc_scatter_x3(a.gc_dtab + (long)l * 64, a.gc_ld, DVs, DVg, w, lane, 32, gc_starts, gc_pid);
      XSTAMP(4);
      // 6. dSIG / dGATE partials of ALL four tiles t (0 sig·prev, 1 sig·cur, 2 gate·prev, 3
      //    gate·cur) over this wave's own 32 positions: A[i=in][k=pos] = X[pos][in], B[k][j=o] =
      //    DV[pos][o], k-step s: p = 32w + 16s + 2j + h (the lane halves read rows of opposite
      //    parity).  Every X and DV value is split once per layer (one tile per wave over all 128
      //    positions split each twice); the four waves' partials are summed through LDS at the end.
      floatx16 accT[4];
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
        for (int q = 0; q < 16; ++q) accT[t4][q] = 0.f;
      {
        const float* isrc = a.bimg + (long)(l > 0 ? l - 1 : 0) * BIMG_F + lane * 4;
        // both k-steps' operands are read before the DMA issue (its asm is a compiler barrier for
        // LDS reads), so that their latency is exposed once
        float xp[2][8], xc[2][8], ds[2][8], dg[2][8];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int p = 32 * w + 16 * s2 + 2 * j + h;
            xp[s2][j] = Xp[CONF(16) ? p * 32 : p * 32 + pi];
            xc[s2][j] = Xc[CONF(16) ? p * 32 : p * 32 + pi];
            ds[s2][j] = DVs[CONF(32) ? p * 32 : swz(p, pi)];
            dg[s2][j] = DVg[CONF(32) ? p * 32 : swz(p, pi)];
          }
        XSTAMP(8);
        if (l > 0) {   // image pieces w, w+4, ... (30 of 1 KiB)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int pc = w + 4 * i;
            if (pc < BX_F / 256 && !CONF(1024)) dma16(isrc + pc * 256, IMG + pc * 256);
          }
          load_regs(l - 1);
        }
        XSTAMP(9);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 fxp[3], fxc[3], fds[3], fdg[3];
          split8(floatx4{xp[s2][0], xp[s2][1], xp[s2][2], xp[s2][3]}, floatx4{xp[s2][4], xp[s2][5], xp[s2][6], xp[s2][7]}, fxp);
          split8(floatx4{ds[s2][0], ds[s2][1], ds[s2][2], ds[s2][3]}, floatx4{ds[s2][4], ds[s2][5], ds[s2][6], ds[s2][7]}, fds);
          accT[0] = mfma_x3(fxp, fds, accT[0]);
          split8(floatx4{xc[s2][0], xc[s2][1], xc[s2][2], xc[s2][3]}, floatx4{xc[s2][4], xc[s2][5], xc[s2][6], xc[s2][7]}, fxc);
          accT[1] = mfma_x3(fxc, fds, accT[1]);
          split8(floatx4{dg[s2][0], dg[s2][1], dg[s2][2], dg[s2][3]}, floatx4{dg[s2][4], dg[s2][5], dg[s2][6], dg[s2][7]}, fdg);
          accT[2] = mfma_x3(fxp, fdg, accT[2]);
          accT[3] = mfma_x3(fxc, fdg, accT[3]);
          if (s2 == 0) XSTAMP(10);
        }
      }
      XSTAMP(5);
      // 7. dRES quarter of wave w (16x16: z channels 16(w>>1).., res out 16(w&1)..) over all LP
      //    positions on v_mfma_f32_16x16x4_f32 (K = 2048 flop/pos is too little to pay for
      //    splitting): A[i=c][k=pos] = z[pos][c], B[k][j=o] = g[pos][o]; k = lane>>4
      floatx4 accR = {0.f, 0.f, 0.f, 0.f};
      {
        const int i16 = lane & 15, kg = lane >> 4, cz = 16 * (w >> 1) + i16, og = 16 * (w & 1) + i16;
#pragma unroll
        for (int c8 = 0; c8 < LP / 32; ++c8) {
          float za[8], ga[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int p = 32 * c8 + 4 * j + kg;
            za[j] = ZT[CONF(64) ? p * 32 : p * 32 + cz];
            ga[j] = G[CONF(128) ? p * 32 : swz(p, og)];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 8; ++j) accR = __builtin_amdgcn_mfma_f32_16x16x4f32(za[j], ga[j], accR, 0, 0, 0);
        }
      }
      XSTAMP(11);
      // 8. bias partials (column sums of DV and G) and the slab
      float* slab = a.slab + ((long)l * ntiles + tile) * SLAB;
      //    (wave 0: DVs, 1: DVg, 2: G; lane = (row class pc, 4-column group c4), rows pc + 8p:
      //    each 16-lane b128 read group then covers both bank halves, conflict-free under swz)
      if (tid < 192) {
        const int c4 = (lane & 7) * 4, pc = lane >> 3;
        const float* pl = w == 0 ? DVs : w == 1 ? DVg : G;
        floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 16; ++p) s4 += *(const floatx4*)(pl + (CONF(256) ? p * 32 : swz(pc + 8 * p, c4)));
        *(floatx4*)(part + pc * 96 + 32 * w + c4) = s4;
      }
      {
        const int i16 = lane & 15, kg = lane >> 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) slab[4096 + (16 * (w >> 1) + 4 * kg + q) * 32 + 16 * (w & 1) + i16] = accR[q];
      }
      __syncthreads();   // every read of Xp/Xc/ZT/DV/G of this layer is done; part complete
      if (tid < 96) {
        float s1 = 0.f;
#pragma unroll
        for (int pc = 0; pc < 8; ++pc) s1 += part[pc * 96 + tid];
        slab[5120 + tid] = s1;
      }
      XSTAMP(12);
      // dSIG / dGATE: partial of tile t to slot (wave, t) of Xp..DVs (64 KiB, dead until the next
      // layer's G-build barrier), lane-linear in accumulator order; wave w sums tile w over waves
      {
        float* SCR = Xp;
        const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *(floatx4*)(SCR + (wu * 4 + t4) * 1024 + (g * 64 + lane) * 4) =
                floatx4{accT[t4][4 * g], accT[t4][4 * g + 1], accT[t4][4 * g + 2], accT[t4][4 * g + 3]};
        __syncthreads();
        XSTAMP(13);
        floatx16 accW;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          floatx4 v[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) v[s4] = *(const floatx4*)(SCR + (CONF(512) ? (s4 * 4 + wu) * 1024 : (s4 * 4 + wu) * 1024 + (g * 64 + lane) * 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) accW[4 * g + e] = (v[0][e] + v[1][e]) + (v[2][e] + v[3][e]);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) slab[w * 1024 + acc_row(q, h) * 32 + pi] = accW[q];
      }
      XSTAMP(6);
    }
#undef XSTAMP
  }
}

// ---- backward chain, 16-position waves (round 4) --------------------------------------------
// chain_bwd16_kernel<NW, TR>: chain_bwd_x3_kernel's layer walk, hand-off protocol, images and slab
// layout with 16 positions per wave and NW waves per block (tile TP = 16·NW: NW = 8 puts two
// waves on each SIMD).  Lane = (j = lane & 15: the wave's position, g = lane >> 4); two channel
// layouts per lane (q0 = 2(g >> 1), h = g & 1):
//   N  (x / g / out_a / out_c0): block xb register r = channel 16xb + 4g + r;
//   Zl (dz / z / σ / dv, the forward's z layout): block b register r = channel 8(q0 + b) + 4h + r.
//  * dz = dZ + RES·g on 16x16x32 bf16 splits (round 5; 16 f32 16x16x4 MFMAs before): A row i of
//    block b = z channel ch16(b, i) from the RX image, k = 8g + e = g's channel 16(e >> 2) + 4g +
//    (e & 3), i.e. the lane's two N-layout g registers split as they are;
//  * dx = W·dv on 16x16x32 bf16 splits, k-step S = sig / gate: the lane's 8 dv values of kind S
//    (Zl blocks 0, 1) are exactly the backward image's k order kk = 32S + 8g + e (WD unchanged);
//  * dSIG / dGATE: wave w takes weight-gradient tile w & 3 (2·kind + tap) over positions
//    [(w >> 2)·TP/NH, +TP/NH) (NH = NW/4 position halves) on 32x32x16 bf16 splits (k = 16
//    positions), and dRES quarter w & 3 over the same positions on 16x16x4 f32; with NH = 2 the
//    two halves' partials are summed through LDS by waves 0-3.
// LDS rows: Xp / Xc / ZT unpadded (LDS-DMA), DVs / DVg / G / OC padded to XS = 36 floats (the
// b128 own-row writes of 16 consecutive rows fall on 16 distinct bank groups).
// WG = false (round 6): the weight gradients leave the chain.  Per layer a tile runs only the
// dependent path (G build, dz / dv, dx, publish) and exports the rows the weight gradients need:
// DV (k-blocked [2L][Mp][32], as the LC products read it) and G = dx_{l+1} ([L][Mp][32]);
// layer_wgrad_kernel forms dSIG / dGATE / dRES / the biases (and the GC sums) from them over all
// positions of a layer.  No x / z DMA, no slab, LDS = image + G + OC.
template <int NW>
constexpr int cb16_lds() { return B16IMG_F + 3 * 16 * NW * 32 + 4 * 16 * NW * XS + 8 * 96; }
template <int NW>
constexpr int cb16_lds_nowg() { return B16IMG_F + 2 * 16 * NW * XS; }
static_assert(cb16_lds<8>() * 4 + 16 <= 160 * 1024, "chain bwd16 LDS");
static_assert(4 * 1280 <= 3 * 128 * 32, "bwd16: the partial scratch (waves 4-7) must fit in Xp | Xc | ZT");

// GC rows of a wave whose 16 positions are not one voice: dv column sums per run of equal ids,
// one atomic per run and column (as gc_scatter_x3, 16 positions)
LBWN_DEV void gc_scatter16(float* gtab, long ld, const float* DVs, const float* DVg, int w, int lane, int Cd,
                           unsigned starts, int pid) {
  const int o = lane, oc = o & 31;
  const float* pl = o < 32 ? DVs : DVg;
  const int col = o < 32 ? oc : Cd + oc;
  unsigned rest = starts;
  while (rest) {   // wave-uniform
    const int p0 = __ffs(rest) - 1;
    rest &= rest - 1;
    const int p1 = rest ? __ffs(rest) - 1 : 16;
    const int id = __shfl(pid, p0);
    if (id < 0) continue;   // positions past T
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += pl[(16 * w + p) * XS + oc];
    if (oc < Cd) atomicAdd(gtab + (long)id * ld + col, s);
  }
}

template <int NW, bool TR, bool WG>
__global__ __launch_bounds__(64 * NW) void chain_bwd16_kernel(ChainBK a) {
  constexpr int TP = 16 * NW, NT = 64 * NW, NH = NW / 4, PH = TP / NH;   // PH: positions per half
  constexpr int NR = TP * 8 / NT;                                        // float4 per thread of a tile (2)
  __shared__ __attribute__((aligned(16))) float sm[WG ? cb16_lds<NW>() : cb16_lds_nowg<NW>()];
  __shared__ int s_fail;
  float* IMG = sm;
  const unsigned short* WD = (const unsigned short*)IMG;
  const unsigned short* RX = WD + BD_US;
  // WG: Xp | Xc | ZT | DVs | DVg | G | OC | part;  !WG: G | OC
  float* Xp = IMG + B16IMG_F;
  float* Xc = Xp + TP * 32;
  float* ZT = Xc + TP * 32;
  float* DVs = ZT + TP * 32;
  float* DVg = DVs + TP * XS;
  float* G = WG ? DVg + TP * XS : IMG + B16IMG_F;
  float* OC = G + TP * XS;
  float* part = OC + TP * XS;   // [8][96] bias partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4, q0 = 2 * (g >> 1), h = g & 1;
  const int r = 16 * w + i16;
  const int tps = (a.T + TP - 1) / TP, ntiles = a.B * tps;
  const int oc_bytes = (int)std::min<long>(a.ocls * 4, 0x7fffffffL);
  if (tid == 0) s_fail = 0;
  const int first = chain_first(a.xcd);
  for (int it = first; it < ntiles; it += gridDim.x) {
    const int tile = ntiles - 1 - it;
    const int b = tile / tps, tt = tile % tps, t0 = tt * TP;
    const int t = t0 + r;
    const bool valid = t < a.T;
    const long mb = (long)b * a.T, m = mb + t, mc = mb + min(t, a.T - 1);
    const long sb = (long)b * (a.H + a.T) * 32;
    const int myid = (WG && a.gc_tab && valid) ? a.ids[m] : 0;
    const int tile_id = (WG && a.gc_tab) ? a.ids[mb + t0] : 0;
    // (!WG: the GC sums and tile ids come from layer_wgrad_kernel)
    const bool tile_uni = WG ? __syncthreads_and(!valid || myid == tile_id) : true;
    if (WG && a.tile_gid && tid == 0) a.tile_gid[tile] = tile_uni ? tile_id : -1;
    // this wave's id runs over its 16 positions (lanes j of the first group), -1 past T
    const int gc_pid = valid ? myid : -1;
    const int gc_prev = WG ? __shfl(gc_pid, max(lane - 1, 0) & 15) : 0;
    const unsigned gc_starts = WG ? (unsigned)(__ballot(g == 0 && (i16 == 0 || gc_pid != gc_prev)) & 0xffffull) : 0u;
    // per-layer rows of this lane's position (Zl channels): dZ, z, σ, issued a layer ahead
    // (buffer loads: a per-layer scalar base and one 32-bit lane offset per array, instead of three
    // 64-bit lane addresses held across the layer loop; the launcher checks the byte ranges)
    floatx4 dzr[2], zr[2], sgr[2];
    const int o_sg = (int)(sg_off(mc, q0, h) * 4), o_z = (int)((mc * a.lddz + 8 * q0 + 4 * h) * 4);
    auto load_regs = [&](int l) {
      const __amdgpu_buffer_rsrc_t rdz = __builtin_amdgcn_make_buffer_rsrc((void*)(a.DZ + l * a.dzls), (short)0, 0x7fffffff, BUF_DW3);
      const __amdgpu_buffer_rsrc_t rsg = __builtin_amdgcn_make_buffer_rsrc((void*)(a.SG + (long)l * a.sgls), (short)0, 0x7fffffff, BUF_DW3);
      const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(a.Zf + (long)l * 32), (short)0, 0x7fffffff, BUF_DW3);
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {   // q0 + 1: the next 8-channel group (sg_off + 256 floats, z + 8)
        dzr[bb] = __builtin_amdgcn_raw_buffer_load_b128(rdz, o_sg + 1024 * bb, 0, 0);
        zr[bb] = __builtin_amdgcn_raw_buffer_load_b128(rz, o_z + 32 * bb, 0, 0);
        sgr[bb] = __builtin_amdgcn_raw_buffer_load_b128(rsg, o_sg + 1024 * bb, 0, 0);
      }
    };
    auto dma_image = [&](int l) {
      const float* src = a.bimg + (long)l * BIMG_F + lane * 4;
      for (int i = w; i < B16IMG_F / 256; i += NW) dma16(src + (i < BD_PC ? i : i - BD_PC + RX_GPC) * 256, IMG + i * 256);
    };
    __syncthreads();  // previous tile's LDS use done
    dma_image(a.L - 1);
    load_regs(a.L - 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    floatx4 oa[2];  // out_a of layer l+1, own row (N layout)
    oa[0] = oa[1] = floatx4{0.f, 0.f, 0.f, 0.f};
    const bool trc = a.trace && (int)blockIdx.x == a.trace_blk && tid == 0 && it == first;
#define XSTAMP(i) if (TR && trc) a.trace[16 * l + (i)] = clock64()
    // the producer's out_c0 rows for the next layer's G build, loaded in this layer's tail (after
    // the weight-gradient products, when the producer published long ago): its flag wait and
    // load latency overlap the bias sums and slab stores instead of opening the next layer
    floatx4 gl[NR];
    floatx4 gx_keep[2], dvs_keep[2], dvg_keep[2];   // !WG: this layer's export rows
    for (int l = a.L - 1; l >= 0; --l) {
      XSTAMP(0);
      const int d = 1 << (l % a.nbl);
      const int dn = (l + 1 < a.L) ? 1 << ((l + 1) % a.nbl) : 0;
      // 1. G = dx_{l+1} rows: out_c0_{l+1}[t + dn] (own OC / the producer's rows, gl) + out_a
      if (dn) {
        XSTAMP(7);
        floatx4 go[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int e = tid + NT * i, sr = (e >> 3) + dn, c4 = (e & 7) * 4;
          go[i] = *(const floatx4*)(OC + min(sr, TP - 1) * XS + c4);
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int e = tid + NT * i, row = e >> 3, c4 = (e & 7) * 4, sr = row + dn, ts = t0 + sr;
          floatx4 v = sr < TP ? go[i] : gl[i];
          if (ts >= a.T) v = floatx4{0.f, 0.f, 0.f, 0.f};
          *(floatx4*)(G + row * XS + c4) = v;
        }
        XSTAMP(14);
        // lands this wave's part of the weight image (DMA'd during the last layer) and the
        // prefetched rows; the barrier then covers every wave's part (!WG: not the 6 export
        // stores issued after them)
        if (WG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        XSTAMP(15);
        __syncthreads();
      }
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) asm volatile("" ::"v"(dzr[bb]), "v"(zr[bb]), "v"(sgr[bb]));
      const float* xl = a.X + (long)l * a.xls + sb;
      // this layer's x rows (x[t-d] | x[t]) and z rows by LDS-DMA into Xp / Xc / ZT, 8 rows per piece
      auto dma_rows3 = [&](int k) {
        const int row = 8 * k + (lane >> 3), c4 = (lane & 7) * 4;
        const int trow = min(t0 + row, a.T - 1);
        dma16(xl + (long)(a.H + trow - d) * 32 + c4, Xp + 8 * k * 32);
        dma16(xl + (long)(a.H + trow) * 32 + c4, Xc + 8 * k * 32);
        dma16(a.Zf + (mb + trow) * a.lddz + (long)l * 32 + c4, ZT + 8 * k * 32);
      };
      XSTAMP(1);
      floatx4 gv[2];
#pragma unroll
      for (int xb = 0; xb < 2; ++xb) {   // own row: + out_a (the top layer writes it, g = 0)
        float* gp = G + r * XS + 16 * xb + 4 * g;
        floatx4 v = dn ? *(const floatx4*)gp : floatx4{0.f, 0.f, 0.f, 0.f};
        v += oa[xb];
        gv[xb] = v;
        if (WG) *(floatx4*)gp = v;
      }
      // 2. dz = dZ + RES·g on the bf16 cores: one 32-deep k-step of six split products per block
      //    bb (A row i = z channel ch16(bb, i) of RX, k = 8g + e = the lane's g registers in order)
      floatx4 dz[2];
      {
        bf16x8 gb[3];
        split8(gv[0], gv[1], gb);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          bf16x8 rx[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) rx[p] = *(const bf16x8*)(RX + ch16(bb, i16) * RX_ROW + 32 * p + 8 * g);
          dz[bb] = mfma16x3(rx, gb, valid ? dzr[bb] : floatx4{0.f, 0.f, 0.f, 0.f});
          // x / z rows of this layer: pieces k = w, w + NW, ... (3·TP/8 rows of 8 over the block)
#pragma unroll
          for (int k2 = 0; k2 < TP / 8 / NW / 2 + 1; ++k2) {
            const int k = w + NW * (2 * k2 + bb);
            if (WG && k < TP / 8) dma_rows3(k);
          }
        }
      }
      // 3. dv from z and σ: tanh = z/σ (σ = 0 only where dv is 0 anyway)
      floatx4 dvs[2], dvg[2];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float zz = zr[bb][e], sg = sgr[bb][e];
          const float th = sg > 1e-30f ? zz * __builtin_amdgcn_rcpf(sg) : 0.f;
          dvs[bb][e] = dz[bb][e] * sg * (1.f - th * th);
          dvg[bb][e] = dz[bb][e] * zz * (1.f - sg);
        }
      {
        // DV export: rows (layer l at columns l·64) or k-blocked (a.dvks: [L·2][Mp][32] chunks)
        float* dvo = (a.dv_out && valid)
                         ? a.dv_out + (a.dvks ? 2L * l * a.dvks + m * 32 : m * a.lddv + (long)l * 64) : nullptr;
        const long dgo = a.dvks ? a.dvks : 32;   // gate half
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int c = 8 * (q0 + bb) + 4 * h;
          if (WG) {
            *(floatx4*)(DVs + r * XS + c) = dvs[bb];
            *(floatx4*)(DVg + r * XS + c) = dvg[bb];
          }
          if (WG && dvo) {
            *(floatx4*)(dvo + c) = dvs[bb];
            *(floatx4*)(dvo + dgo + c) = dvg[bb];
          }
        }
      }
      // !WG: the next layer's dZ / z / σ rows now (this layer's are consumed)
      if (!WG && l > 0) load_regs(l - 1);
      XSTAMP(2);
      // 4. dx on the bf16 cores: out_a = g + W1·dv, out_c0 = W0·dv (k-steps S = 0 sig, 1 gate)
      floatx4 acc_a[2] = {gv[0], gv[1]}, acc_c[2];
      acc_c[0] = acc_c[1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int S = 0; S < 2; ++S) {
        bf16x8 fa[2][3], fc[2][3];
#pragma unroll
        for (int xb = 0; xb < 2; ++xb)
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            fa[xb][p] = *(const bf16x8*)(WD + (32 + 16 * xb + i16) * XW_ROW + 64 * p + 32 * S + 8 * g);
            fc[xb][p] = *(const bf16x8*)(WD + (16 * xb + i16) * XW_ROW + 64 * p + 32 * S + 8 * g);
          }
        bf16x8 bx[3];
        if (S == 0) split8(dvs[0], dvs[1], bx);
        else split8(dvg[0], dvg[1], bx);
#pragma unroll
        for (int xb = 0; xb < 2; ++xb) {
          acc_a[xb] = mfma16x3(fa[xb], bx, acc_a[xb]);
          acc_c[xb] = mfma16x3(fc[xb], bx, acc_c[xb]);
        }
      }
      {
        const __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)l * a.ocls, (short)0, oc_bytes, BUF_DW3);
        const bool pub = l > 0 && valid && r < min(d, TP);
#pragma unroll
        for (int xb = 0; xb < 2; ++xb) {
          *(floatx4*)(OC + r * XS + 16 * xb + 4 * g) = acc_c[xb];
          if (pub) __builtin_amdgcn_raw_buffer_store_b128(acc_c[xb], rw, (int)((m * 32 + 16 * xb + 4 * g) * 4), 0, 16);
        }
      }
      if (l == 0 && valid) {
#pragma unroll
        for (int xb = 0; xb < 2; ++xb) {
          *(floatx4*)(a.dx0_a + m * 32 + 16 * xb + 4 * g) = acc_a[xb];
          *(floatx4*)(a.dx0_c + m * 32 + 16 * xb + 4 * g) = acc_c[xb];
        }
      }
      oa[0] = acc_a[0];
      oa[1] = acc_a[1];
      if (!WG) {   // kept for the exports after the publish
        gx_keep[0] = gv[0]; gx_keep[1] = gv[1];
        dvs_keep[0] = dvs[0]; dvs_keep[1] = dvs[1];
        dvg_keep[0] = dvg[0]; dvg_keep[1] = dvg[1];
      }
      XSTAMP(3);
      // 5. publish out_c0_l (the drain also lands this layer's x / z DMA pieces)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // DV, G, OC, Xp/Xc/ZT complete; the weight image is dead
      if (tid == 0 && l > 0) publish_flag(a.flags + tile, (unsigned)(a.L - l));
      if (!WG) {
        XSTAMP(4);
        if (l > 0) {
          // the next layer's image (this layer's dx was its last reader), then the producer of the
          // next layer's G rows: each wave polls its flag (lane 0) and loads its own rows, so no
          // block barrier sits between the publish and the next layer's G build
          dma_image(l - 1);
          const int pn = tt + max(1, d / TP);
          if (pn < tps) {
            if (lane == 0 && !s_fail) {
              if (!wait_flag_ge(a.flags + (long)b * tps + pn, (unsigned)(a.L - l), a.status, 2u)) s_fail = 1;
            }
            __builtin_amdgcn_wave_barrier();
          }
          XSTAMP(5);
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)l * a.ocls, (short)0, oc_bytes, BUF_DW3);
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            const int e = tid + NT * i, c4 = (e & 7) * 4;
            const int ts = min(t0 + (e >> 3) + d, a.T - 1);
            gl[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((mb + ts) * 32 + c4) * 4), 0, 16);
          }
        }
        // the exports for the weight gradients (G = dx_{l+1} rows, DV) only now, behind the G row
        // loads: the publish drain did not wait for them, and the next G build waits only for what
        // was issued before them (vmcnt(6)).  Every lane stores (a past-T lane at an offset past
        // the record: the store is dropped), so each wave issues exactly 6 of them.
        {
          const int nrec = (int)std::min<long>((long)a.B * a.T * 128, 0x7fffffffL);
          const int ok = valid ? (int)(m * 128) : 0x7ffffff0;
          const __amdgpu_buffer_rsrc_t rgx = __builtin_amdgcn_make_buffer_rsrc(a.gx + l * a.gxls, (short)0, nrec, BUF_DW3);
          const __amdgpu_buffer_rsrc_t rvs = __builtin_amdgcn_make_buffer_rsrc(a.dv_out + 2L * l * a.dvks, (short)0, nrec, BUF_DW3);
          const __amdgpu_buffer_rsrc_t rvg = __builtin_amdgcn_make_buffer_rsrc(a.dv_out + (2L * l + 1) * a.dvks, (short)0, nrec, BUF_DW3);
#pragma unroll
          for (int xb = 0; xb < 2; ++xb) __builtin_amdgcn_raw_buffer_store_b128(gx_keep[xb], rgx, ok + (16 * xb + 4 * g) * 4, 0, 0);
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) {
            const int cz = (8 * (q0 + bb) + 4 * h) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(dvs_keep[bb], rvs, ok + cz, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(dvg_keep[bb], rvg, ok + cz, 0, 0);
          }
        }
        XSTAMP(6);
        continue;
      }
      if (a.gc_dtab && !tile_uni) gc_scatter16(a.gc_dtab + (long)l * 64, a.gc_ld, DVs, DVg, w, lane, 32, gc_starts, gc_pid);
      XSTAMP(4);
      // 6. dSIG / dGATE tile t4 = w & 3 (2·kind + tap) over this wave's position half:
      //    A[i = in][k = pos] = X_tap[pos][in], B[k = pos][j = o] = DV_kind[pos][o]
      const int t4 = w & 3, p0 = (w >> 2) * PH;
      floatx16 accT;
#pragma unroll
      for (int q = 0; q < 16; ++q) accT[q] = 0.f;
      {
        const float* XA = (t4 & 1) ? Xc : Xp;
        const float* DB = (t4 & 2) ? DVg : DVs;
        const int pi = lane & 31, hh = lane >> 5;
        float xa[PH / 16][8], db[PH / 16][8];
#pragma unroll
        for (int s2 = 0; s2 < PH / 16; ++s2)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int p = p0 + 16 * s2 + 8 * hh + e;
            xa[s2][e] = XA[p * 32 + pi];
            db[s2][e] = DB[p * XS + pi];
          }
        XSTAMP(8);
        if (l > 0) {   // the next layer's image and rows, behind this layer's operand reads
          dma_image(l - 1);
          load_regs(l - 1);
        }
        XSTAMP(9);
#pragma unroll
        for (int s2 = 0; s2 < PH / 16; ++s2) {
          bf16x8 fx[3], fd[3];
          split8(floatx4{xa[s2][0], xa[s2][1], xa[s2][2], xa[s2][3]}, floatx4{xa[s2][4], xa[s2][5], xa[s2][6], xa[s2][7]}, fx);
          split8(floatx4{db[s2][0], db[s2][1], db[s2][2], db[s2][3]}, floatx4{db[s2][4], db[s2][5], db[s2][6], db[s2][7]}, fd);
          accT = mfma_x3(fx, fd, accT);
          if (s2 == 0) XSTAMP(10);
        }
      }
      XSTAMP(5);
      // 7. dRES quarter t4 (16x16: z channels 16(t4>>1).., res out 16(t4&1)..) over the same
      //    positions on v_mfma_f32_16x16x4_f32: A[i=c][k=pos] = z[pos][c], B[k=pos][j=o] = g[pos][o]
      floatx4 accR = {0.f, 0.f, 0.f, 0.f};
      {
        const int cz = 16 * (t4 >> 1) + i16, og = 16 * (t4 & 1) + i16;
#pragma unroll
        for (int c8 = 0; c8 < PH / 32; ++c8) {
          float za[8], ga[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int p = p0 + 32 * c8 + 4 * e + g;
            za[e] = ZT[p * 32 + cz];
            ga[e] = G[p * XS + og];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < 8; ++e) accR = __builtin_amdgcn_mfma_f32_16x16x4f32(za[e], ga[e], accR, 0, 0, 0);
        }
      }
      XSTAMP(11);
      // 8. bias partials (column sums of DVs, DVg, G: waves 0-2; lane = (row class pc, 4-column
      //    group c4), rows pc + 8p)
      float* slab = a.slab + ((long)l * ntiles + tile) * SLAB;
      if (w < 3) {
        const int c4 = (lane & 7) * 4, pc = lane >> 3;
        const float* pl = w == 0 ? DVs : w == 1 ? DVg : G;
        floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < TP / 8; ++p) s4 += *(const floatx4*)(pl + (pc + 8 * p) * XS + c4);
        *(floatx4*)(part + pc * 96 + 32 * w + c4) = s4;
      }
      // the next layer's producer: its flag (published after its dx of this layer, half a layer
      // ago) and then its out_c0 rows, loaded after the barrier below
      const int pn = tt + max(1, d / TP);
      if (l > 0 && pn < tps && tid == 0 && !s_fail) {
        if (!wait_flag_ge(a.flags + (long)b * tps + pn, (unsigned)(a.L - l), a.status, 2u)) s_fail = 1;
      }
      __syncthreads();   // every read of Xp/Xc/ZT/DV/G of this layer is done; part complete; the flag seen
      {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(a.ocg + (long)l * a.ocls, (short)0, oc_bytes, BUF_DW3);
#pragma unroll
        for (int i = 0; i < NR; ++i) {   // (l = 0: a dead load of valid rows)
          const int e = tid + NT * i, c4 = (e & 7) * 4;
          const int ts = min(t0 + (e >> 3) + d, a.T - 1);
          gl[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((mb + ts) * 32 + c4) * 4), 0, 16);
        }
      }
      if (tid < 96) {
        float s1 = 0.f;
#pragma unroll
        for (int pc = 0; pc < 8; ++pc) s1 += part[pc * 96 + tid];
        slab[5120 + tid] = s1;
      }
      XSTAMP(12);
      // weight-gradient partials to the slab: with two position halves, each wave parks its
      // partials lane-linear in Xp.. (dead until the next layer's G-build barrier) and waves 0-3
      // sum halves 0 + 1 of their tile / quarter in a fixed order
      if (NH == 1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) slab[t4 * 1024 + acc_row(q, lane >> 5) * 32 + (lane & 31)] = accT[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) slab[4096 + (16 * (t4 >> 1) + 4 * g + q) * 32 + 16 * (t4 & 1) + i16] = accR[q];
      } else {
        // (only waves 4-7 park theirs: waves 0-3 add their own half from registers, in the same order)
        if (w >= 4) {
          float* SCR = Xp + (w - 4) * 1280;
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
            *(floatx4*)(SCR + (q4 * 64 + lane) * 4) = floatx4{accT[4 * q4], accT[4 * q4 + 1], accT[4 * q4 + 2], accT[4 * q4 + 3]};
          *(floatx4*)(SCR + 1024 + lane * 4) = accR;
        }
        __syncthreads();
        XSTAMP(13);
        if (w < 4) {
          const float* S1 = Xp + w * 1280;
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const floatx4 v = floatx4{accT[4 * q4], accT[4 * q4 + 1], accT[4 * q4 + 2], accT[4 * q4 + 3]} +
                              *(const floatx4*)(S1 + (q4 * 64 + lane) * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) slab[w * 1024 + acc_row(4 * q4 + e, lane >> 5) * 32 + (lane & 31)] = v[e];
          }
          const floatx4 v = accR + *(const floatx4*)(S1 + 1024 + lane * 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) slab[4096 + (16 * (w >> 1) + 4 * g + q) * 32 + 16 * (w & 1) + i16] = v[q];
        }
      }
      XSTAMP(6);
    }
#undef XSTAMP
  }
}

// Sum every layer's slab partials: grid (column groups, L).
// At most 32 VGPRs (22 at this writing, -Rpass-analysis=kernel-resource-usage): it runs on the side stream beside dSKIP's A-in-registers GEMM
// blocks (2 waves of 240 VGPRs per SIMD leave 32), so it must fit in what they leave free or it
// waits for them.  Parts p8, p8 + 8, ... in order (the order of slab_group_prefetch/finish).
__global__ __launch_bounds__(256) void layer_reduce_all_kernel(
    RedK a, long slab_layer, long dsig_l, long dres_l, long db_l) {
  __shared__ float scratch[256];
  const int l = blockIdx.y, tid = threadIdx.x;
  RedK k = a;
  k.slab = a.slab + l * slab_layer;
  k.dsig = a.dsig + l * dsig_l;
  k.dgate = a.dgate + l * dsig_l;
  k.dres = a.dres + l * dres_l;
  k.dbsig = a.dbsig ? a.dbsig + l * db_l : nullptr;
  k.dbgate = a.dbgate ? a.dbgate + l * db_l : nullptr;
  k.dbres = a.dbres ? a.dbres + l * (long)a.Cr : nullptr;
  const int c = blockIdx.x * 32 + (tid & 31), p8 = tid >> 5, cc = min(c, SLAB - 1);
  float s = 0.f;
  // buffer loads: one 32-bit offset per load instead of a 64-bit address (the VGPR budget above);
  // parts past nparts read past the record (0, and the zero is never added: nparts bounds it)
  const int st = (int)k.stride;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(k.slab), (short)0, (int)std::min<long>((long)k.nparts * st * 4, 0x7fffffffL), 0x00020000);
  for (int p0 = p8; p0 < k.nparts; p0 += 64) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, ((p0 + 8 * i) * st + cc) * 4, 0, 0));
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (p0 + 8 * i < k.nparts) ? v[i] : 0.f;
  }
  scratch[tid] = s;
  __syncthreads();
  if (tid < 32 && c < SLAB) {
    float tot = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) tot += scratch[j * 32 + tid];
    slab_store(k, c, tot);
  }
}

// ---- residual-stack weight gradients over all positions (round 6) --------------------------
// layer_wgrad_kernel<GC>: block (chunk, l) sums, over the positions of tpc consecutive chain tiles
// (128 positions each, tile = b·tps + tt as in the chains), the weight-gradient partials of layer
// l that chain_bwd16_kernel<.., true> forms per tile inside the chain (tmodel.py:136-148 conv,
// :171-184 residual, differentiated at :354-358):
//   dSIG / dGATE[tap][in][o] = Σ_t x_l[t - (1-tap)·d][in] · dv_{sig|gate}[t][o],
//   dRES[c][o] = Σ_t z_l[t][c] · G[t][o],  biases = Σ_t dv_sig, dv_gate, G,
// from the rows the chain exported (DV k-blocked [2L][Mp][32], G [L][Mp][32]) and the forward's x
// and z rows.  Products on 32x32x16 bf16 splits (six products, f32 accumulate),
// k = 16 positions: lane (c = lane & 31, kh = lane >> 5) holds positions 8kh..8kh+7 of channel c
// for both operands, loaded as scalars straight from the position-major rows (two 128-B runs per
// instruction), the next k-step's 48 values in flight behind this one's MFMAs.  Wave w takes
// tiles w, w + 4, ... of the chunk; the four waves' partials meet in LDS in a fixed order and the
// block writes one slab partial [l][chunk][SLAB] in the layout layer_reduce_all_kernel reads.
// GC: per tile, the wave tests the voice ids; a uniform tile's dv column sums go to gcs
// [l][tile][64] for gc_tile_sum_kernel (deterministic), a mixed tile's runs are added to the GC
// table with atomics, as the chains do.
struct WgK {
  const float* X; long xls;       // x_l rows [B][H+T][32] per layer
  const float* Z; long lddz;      // z rows [M][L·32]
  const float* DV; long dvks;     // [2L][Mp][32] (sig chunk 2l, gate chunk 2l+1)
  const float* GX; long gxls;     // [L][Mp][32]
  float* slab; long stride;       // [L][nchunk][stride]
  const int* ids; int* tile_gid; float* gcs; float* gtab; long gc_ld;
  int B, T, H, L, nbl, tps, ntiles, tpc, nchunk;
};

constexpr int WG_TPC_MAX = 64;   // tiles per chunk

template <bool GC>
__global__ __launch_bounds__(256, 2) void layer_wgrad_kernel(WgK a) {
  __shared__ __attribute__((aligned(16))) float scr[3 * SLAB];
  __shared__ int s_gid[WG_TPC_MAX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, kh = lane >> 5;
  const int l = blockIdx.y, ch = blockIdx.x;
  const int d = 1 << (l % a.nbl);
  const int tile_beg = ch * a.tpc + w, tile_end = min((ch + 1) * a.tpc, a.ntiles);
  const int nsteps = tile_beg < tile_end ? (tile_end - tile_beg + 3) / 4 * 8 : 0;
  // buffer resources: x[t] and x[t-d] share one lane offset (the tap's base is d rows lower), so
  // do dv_sig, dv_gate and G (one offset per position, three bases)
  const float* xl = a.X + (long)l * a.xls;
  const __amdgpu_buffer_rsrc_t rxc = __builtin_amdgcn_make_buffer_rsrc((void*)xl, (short)0, 0x7fffffff, BUF_DW3);
  const __amdgpu_buffer_rsrc_t rxp = __builtin_amdgcn_make_buffer_rsrc((void*)(xl - 32L * d), (short)0, 0x7fffffff, BUF_DW3);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(a.Z + (long)l * 32), (short)0, 0x7fffffff, BUF_DW3);
  const float* dvl = a.DV + 2L * l * a.dvks;
  const __amdgpu_buffer_rsrc_t rvs = __builtin_amdgcn_make_buffer_rsrc((void*)dvl, (short)0, 0x7fffffff, BUF_DW3);
  const __amdgpu_buffer_rsrc_t rvg = __builtin_amdgcn_make_buffer_rsrc((void*)(dvl + a.dvks), (short)0, 0x7fffffff, BUF_DW3);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(a.GX + (long)l * a.gxls), (short)0, 0x7fffffff, BUF_DW3);
  floatx16 acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
  float bsum[3] = {0.f, 0.f, 0.f};
  // k-step j of this wave: tile tile_beg + 4(j >> 3), 16 positions from 16(j & 7); this lane's 8
  // positions start at t; positions past T are loaded at row T-1 and their dv / G zeroed
  auto pos = [&](int j, int& b, int& t) {
    const int tile = tile_beg + 4 * (j >> 3);
    b = tile / a.tps;
    t = (tile - b * a.tps) * 128 + 16 * (j & 7) + 8 * kh;
  };
  auto load = [&](int j, float (&v)[6][8]) {
    int b, t;
    pos(j, b, t);
    const int mrow = b * a.T, xoff = (b + 1) * a.H * 128;   // x row = m + (b+1)·H
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = mrow + min(t + e, a.T - 1);
      const int om = (m * 32 + c) * 4;
      v[0][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rxp, om, xoff, 0));
      v[1][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rxc, om, xoff, 0));
      v[2][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rz, (int)(((long)m * a.lddz + c) * 4), 0, 0));
      v[3][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rvs, om, 0, 0));
      v[4][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rvg, om, 0, 0));
      v[5][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, om, 0, 0));
    }
  };
  float bt[3] = {0.f, 0.f, 0.f};   // column sums of dv_sig, dv_gate, G over the current tile
  auto compute = [&](int j, float (&v)[6][8]) {
    int b, t;
    pos(j, b, t);
    const int nv = a.T - t;   // valid positions of this lane's 8 (<= 0: none)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e >= nv) v[3][e] = v[4][e] = v[5][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bt[0] += v[3][e];
      bt[1] += v[4][e];
      bt[2] += v[5][e];
    }
    bf16x8 fs[3], fg[3], fx[3];
    split8(floatx4{v[3][0], v[3][1], v[3][2], v[3][3]}, floatx4{v[3][4], v[3][5], v[3][6], v[3][7]}, fs);
    split8(floatx4{v[4][0], v[4][1], v[4][2], v[4][3]}, floatx4{v[4][4], v[4][5], v[4][6], v[4][7]}, fg);
    split8(floatx4{v[0][0], v[0][1], v[0][2], v[0][3]}, floatx4{v[0][4], v[0][5], v[0][6], v[0][7]}, fx);
    acc[0] = mfma_x3(fx, fs, acc[0]);
    acc[2] = mfma_x3(fx, fg, acc[2]);
    split8(floatx4{v[1][0], v[1][1], v[1][2], v[1][3]}, floatx4{v[1][4], v[1][5], v[1][6], v[1][7]}, fx);
    acc[1] = mfma_x3(fx, fs, acc[1]);
    acc[3] = mfma_x3(fx, fg, acc[3]);
    split8(floatx4{v[2][0], v[2][1], v[2][2], v[2][3]}, floatx4{v[2][4], v[2][5], v[2][6], v[2][7]}, fx);
    split8(floatx4{v[5][0], v[5][1], v[5][2], v[5][3]}, floatx4{v[5][4], v[5][5], v[5][6], v[5][7]}, fs);
    acc[4] = mfma_x3(fx, fs, acc[4]);
  };
  // GC: every tile of this wave tested for one voice id before any row load is in flight (the
  // wait for the ids is then not a wait for the prefetched rows); the id or -1 in s_gid
  if (GC) {
    for (int tile = tile_beg; tile < tile_end; tile += 4) {
      const int b = tile / a.tps, t0 = (tile - b * a.tps) * 128;
      const long mb = (long)b * a.T;
      const int i0 = a.ids[mb + min(t0 + lane, a.T - 1)], i1 = a.ids[mb + min(t0 + 64 + lane, a.T - 1)];
      const int id0 = __shfl(i0, 0);
      const int gid = __all(i0 == id0 && i1 == id0) ? id0 : -1;
      if (lane == 0) {
        a.tile_gid[tile] = gid;
        s_gid[tile - ch * a.tpc] = gid;
      }
    }
  }
  // the tile of k-step j is complete: its sums into the totals (and, one voice, to gcs)
  auto close_tile = [&](int j) {
#pragma unroll
    for (int i = 0; i < 3; ++i) bsum[i] += bt[i];
    if (GC) {   // every tile (no branch: gc_tile_sum reads only the one-voice tiles)
      const int tile = tile_beg + 4 * (j >> 3);
      const float g0 = bt[0] + __shfl_xor(bt[0], 32), g1 = bt[1] + __shfl_xor(bt[1], 32);
      float* o = a.gcs + ((long)l * a.ntiles + tile) * 64 + c;
      o[32 * kh] = kh ? g1 : g0;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) bt[i] = 0.f;
  };
  if (nsteps > 0) {
    float va[6][8], vb[6][8];
    load(0, va);
    // a tile's 8 k-steps unrolled (a branch inside the k-step loop cost 112 spilled VGPRs); the
    // next tile's first rows are in flight across the tile boundary; the last prefetch re-loads
    for (int jb = 0; jb < nsteps; jb += 8) {
#pragma unroll
      for (int s2 = 0; s2 < 8; s2 += 2) {
        load(jb + s2 + 1, vb);
        compute(jb + s2, va);
        load(min(jb + s2 + 2, nsteps - 1), va);
        compute(jb + s2 + 1, vb);
      }
      close_tile(jb);
    }
  }
  // GC, tiles of more than one voice (rare): one atomic per run of equal ids, lane = (column c,
  // position half kh), dv re-read from the export
  if (GC) {
    for (int tile = tile_beg; tile < tile_end; tile += 4) {
      if (s_gid[tile - ch * a.tpc] >= 0) continue;
      const int b = tile / a.tps, t0 = (tile - b * a.tps) * 128 + 64 * kh;
      const long mb = (long)b * a.T;
      const float* dvs = dvl + c;
      float s0 = 0.f, s1 = 0.f;
      int cur = -1;
      for (int p = 0; p < 64 && t0 + p < a.T; ++p) {
        const long m = mb + t0 + p;
        const int id = a.ids[m];
        if (id != cur && cur >= 0) {
          atomicAdd(a.gtab + (long)cur * a.gc_ld + (long)l * 64 + c, s0);
          atomicAdd(a.gtab + (long)cur * a.gc_ld + (long)l * 64 + 32 + c, s1);
          s0 = s1 = 0.f;
        }
        cur = id;
        s0 += dvs[m * 32];
        s1 += dvs[a.dvks + m * 32];
      }
      if (cur >= 0) {
        atomicAdd(a.gtab + (long)cur * a.gc_ld + (long)l * 64 + c, s0);
        atomicAdd(a.gtab + (long)cur * a.gc_ld + (long)l * 64 + 32 + c, s1);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) bsum[i] += __shfl_xor(bsum[i], 32);
  // slab index of accumulator register q: tiles t4 = 2·kind + tap at t4·1024, dRES at 4096
  if (w > 0) {
    float* S = scr + (w - 1) * SLAB;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) S[i * 1024 + acc_row(q, kh) * 32 + c] = acc[i][q];
    if (kh == 0) {
      S[5120 + c] = bsum[0];
      S[5152 + c] = bsum[1];
      S[5184 + c] = bsum[2];
    }
  }
  __syncthreads();
  if (w == 0) {
    float* out = a.slab + ((long)l * a.nchunk + ch) * a.stride;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = i * 1024 + acc_row(q, kh) * 32 + c;
        out[k] = ((acc[i][q] + scr[k]) + scr[SLAB + k]) + scr[2 * SLAB + k];
      }
    if (kh == 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int k = 5120 + 32 * i + c;
        out[k] = ((bsum[i] + scr[k]) + scr[SLAB + k]) + scr[2 * SLAB + k];
      }
    }
  }
}

// ---- backward ----------------------------------------------------------------------------
// LDS (112.5 KB, so that one GEMM block of the concurrent weight-gradient stream fits
// beside it on the CU): Xp | Xc | G | IMG | DV.  After the dx step the weight image is dead
// and holds zᵀ (ZT); RED (dRES cross-wave sum, bias partials) reuses Xp once step 5 is done.
constexpr int BWD_LDS = 3 * LP * XS + WIMG + LP * DS;
static_assert(LP * XS <= WIMG, "ZT must fit in the weight image");
static_assert(4 * 1024 <= LP * XS, "RED must fit in Xp");

__global__ __launch_bounds__(256) void layer_bwd_kernel(BwdK a) {
  __shared__ __attribute__((aligned(16))) float sm[BWD_LDS];
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* G = Xc + LP * XS;
  float* Ws = G + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* DV = Ws + WIMG;             // [LP][DS]   dv (sig | gate), position-major
  float* ZT = Ws;                    // [LP][XS]   z, position-major (after step 4)
  float* RED = Xp;                   // 4 × 1024 / [8][96] (after step 5)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;

  floatx16 accW, accR;  // tile w of dSIG/dGATE (w: 0 sig·prev, 1 sig·cur, 2 gate·prev, 3 gate·cur), dRES part
#pragma unroll
  for (int r = 0; r < 16; ++r) { accW[r] = 0.f; accR[r] = 0.f; }
  float bsum = 0.f;  // bias partial: tid<64 dv column, 64..95 g column

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, t0 = (tile % tps) * LP;
    const long mb = (long)b * a.T;
    const float* xb = a.x_in + (long)b * (a.H + a.T) * a.Cr;
    if (tile != (int)blockIdx.x) __syncthreads();  // previous tile's LDS reads done
    stage_image(Ws, a.wpack, tid);
    stage_rows(Xp, xb, t0, -a.d, a.T, a.H, a.Cr, tid);
    stage_rows(Xc, xb, t0, 0, a.T, a.H, a.Cr, tid);
    stage_g(G, a.g_a, a.g_c0, a.g_d, mb, t0, a.T, a.Cr, tid);
    const int t = t0 + 32 * w + pi;
    const bool valid = t < a.T;
    const long m = mb + t;
    // dZ_skip rows (acc layout: channels 8q+4h..+3 per q)
    floatx16 dz;
    if (a.Cd == 32) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 v = *(const floatx4*)(a.dz_skip + (mb + min(t, a.T - 1)) * a.lddz + 8 * q + 4 * h);
        if (!valid) v = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) dz[4 * q + j] = v[j];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = acc_row(r, h);
        dz[r] = (valid && c < a.Cd) ? a.dz_skip[m * a.lddz + c] : 0.f;
      }
    }
    __syncthreads();

    // 1. recompute the gate
    floatx16 acc_s, acc_g;
    if (LBWN_ABL & 4) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc_s[r] = Xc[r]; acc_g[r] = Xp[r]; }
    } else {
      conv_tile(Xp, Xc, Ws, bs, a, m, valid, w, lane, acc_s, acc_g);
    }
    floatx16 th, sg;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      th[r] = tanhf_(acc_s[r]);
      sg[r] = sigmoidf_(acc_g[r]);
    }
    // 2. dzᵀ += RES·gᵀ   (dz[pos][c] = dZ[pos][c] + Σ_o g[pos][o]·RES[c][o])
    const float* gp = G + (32 * w + pi) * XS;
    {
      floatx4 gx[4], rx[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        gx[g] = *(const floatx4*)(gp + 8 * g + 4 * h);
        rx[g] = *(const floatx4*)(Rs + pi * XS + 8 * g + 4 * h);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) dz = mfma32(rx[g][j], gx[g][j], dz);
    }
    // 3. dvᵀ, parked position-major for the weight-grad products
    floatx16 dvs, dvg;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dvs[r] = dz[r] * sg[r] * (1.f - th[r] * th[r]);
      dvg[r] = dz[r] * th[r] * sg[r] * (1.f - sg[r]);
    }
    float* dvrow = DV + (32 * w + pi) * DS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *(floatx4*)(dvrow + 8 * q + 4 * h) = floatx4{dvs[4 * q], dvs[4 * q + 1], dvs[4 * q + 2], dvs[4 * q + 3]};
      *(floatx4*)(dvrow + 32 + 8 * q + 4 * h) = floatx4{dvg[4 * q], dvg[4 * q + 1], dvg[4 * q + 2], dvg[4 * q + 3]};
    }
    // 4. dx: dcurᵀ = W1·dvᵀ (+ g), dprevᵀ = W0·dvᵀ   (rows = in channel)
    floatx16 acc_a, acc_c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 gv = *(const floatx4*)(gp + 8 * q + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc_a[4 * q + j] = gv[j]; acc_c[4 * q + j] = 0.f; }
    }
    {
      floatx4 wv[2][4];  // [buf][w0s, w0g, w1s, w1g]
      auto loadw = [&](int q, int buf) {
        const int ko = 8 * q + 4 * h;
        wv[buf][0] = *(const floatx4*)(Ws + pi * WS + ko);
        wv[buf][1] = *(const floatx4*)(Ws + pi * WS + 32 + ko);
        wv[buf][2] = *(const floatx4*)(Ws + (32 + pi) * WS + ko);
        wv[buf][3] = *(const floatx4*)(Ws + (32 + pi) * WS + 32 + ko);
      };
      loadw(0, 0);
#pragma unroll
      for (int q = 0; q < ((LBWN_ABL & 8) ? 0 : 4); ++q) {
        const int cb = q & 1;
        if (q + 1 < 4) loadw(q + 1, cb ^ 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int s2 = 4 * q + j;
          acc_a = mfma32(wv[cb][2][j], dvs[s2], acc_a);
          acc_c = mfma32(wv[cb][0][j], dvs[s2], acc_c);
          acc_a = mfma32(wv[cb][3][j], dvg[s2], acc_a);
          acc_c = mfma32(wv[cb][1][j], dvg[s2], acc_c);
        }
      }
    }
    if (valid && !(LBWN_ABL & 16)) {
      store_rows16(a.out_a + m * a.Cr, acc_a, a.Cr, h);
      store_rows16(a.out_c0 + m * a.Cr, acc_c, a.Cr, h);
    }
    if (LBWN_ABL & 16) asm volatile("" ::"v"(acc_a[0]), "v"(acc_c[0]), "v"(acc_a[15]), "v"(acc_c[15]));
    __syncthreads();  // DV of every wave visible; nobody reads the weight image any more
    {
      float* zrow = ZT + (32 * w + pi) * XS;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 zv;
#pragma unroll
        for (int j = 0; j < 4; ++j) zv[j] = th[4 * q + j] * sg[4 * q + j];
        *(floatx4*)(zrow + 8 * q + 4 * h) = zv;
      }
    }

    // 5. dSIG/dGATE tile w over all LP positions: A[i=in][k=pos] = X[pos][in], B[k][j=o] = DV[pos][o]
    {
      const float* X = (w & 1) ? Xc : Xp;
      const int oc = (w >> 1) * 32 + pi;
      float xa[2][8], da[2][8];
      auto loadb = [&](int bt, int buf) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int p = 2 * (8 * bt + i) + h;
          xa[buf][i] = X[p * XS + pi];
          da[buf][i] = DV[p * DS + oc];
        }
      };
      loadb(0, 0);
#pragma unroll
      for (int bt = 0; bt < ((LBWN_ABL & 2) ? 0 : LP / 16); ++bt) {
        const int cb = bt & 1;
        if (bt + 1 < LP / 16) loadb(bt + 1, cb ^ 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) accW = mfma32(xa[cb][i], da[cb][i], accW);
      }
    }
    __syncthreads();  // ZT visible; Xp/Xc free for RED
    // 6. dRES part over this wave's 32 positions: A[i=c][k=pos] = z[pos][c], B[k][j=o] = g[pos][o]
    {
      float za[16], ga[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int p = 32 * w + 2 * s2 + h;
        za[s2] = ZT[p * XS + pi];
        ga[s2] = G[p * XS + pi];
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) accR = mfma32(za[s2], ga[s2], accR);
    }
    // bias partials: column sums of DV (64) and G (32) over the tile, 8 position chunks
    {
      float* part = RED;  // [8][96]
      if (tid < 128) {
        const int c4 = (tid & 15) * 4, pc = tid >> 4;
        floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 16; ++p) s4 += *(const floatx4*)(DV + (pc * 16 + p) * DS + c4);
        *(floatx4*)(part + pc * 96 + c4) = s4;
      } else if (tid < 192) {
        const int c4 = ((tid - 128) & 7) * 4, pc = (tid - 128) >> 3;
        floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 16; ++p) s4 += *(const floatx4*)(G + (pc * 16 + p) * XS + c4);
        *(floatx4*)(part + pc * 96 + 64 + c4) = s4;
      }
      __syncthreads();
      if (tid < 96) {
        float s1 = 0.f;
#pragma unroll
        for (int pc = 0; pc < 8; ++pc) s1 += part[pc * 96 + tid];
        bsum += s1;
      }
    }
    // 7. optional dv export (LC grads) and GC table grads
    if (a.dv_out) {
      for (int e = tid; e < LP * 64; e += 256) {
        const int p = e >> 6, o = e & 63, oc = o & 31, tt = t0 + p;
        if (tt < a.T && oc < a.Cd) a.dv_out[(mb + tt) * a.lddv + (o < 32 ? oc : a.Cd + oc)] = DV[p * DS + o];
      }
    }
    if (a.gc_dtab) gc_scatter(a.gc_dtab, a.gc_ld, a.ids + mb, DV, t0, a.T, w, lane, a.Cd, -1);
  }

  // 8. block partial -> slab: tiles 0..3 straight from their wave, dRES summed over waves
  __syncthreads();  // bias partial reads of RED done
  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    slab[w * 1024 + acc_row(r, h) * 32 + pi] = accW[r];
    RED[w * 1024 + acc_row(r, h) * 32 + pi] = accR[r];
  }
  __syncthreads();
  for (int e = tid; e < 1024; e += 256) slab[4096 + e] = ((RED[e] + RED[1024 + e]) + RED[2048 + e]) + RED[3072 + e];
  if (tid < 96) slab[5120 + tid] = bsum;
}

__global__ __launch_bounds__(256) void layer_reduce_kernel(RedK a) {
  __shared__ float scratch[256];
  float pre[RED_PARTS];
  const int ngroups = (SLAB + 31) / 32;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    slab_group_prefetch(a, grp, pre, threadIdx.x);
    slab_group_finish(a, grp, pre, scratch, threadIdx.x);
  }
}

int grid_fwd(const lbwn_layer_args& a) { return std::min(lbwn_layer_nblocks(a.B, a.T), 512); }
int grid_bwd(const lbwn_layer_args& a) { return std::min(lbwn_layer_nblocks(a.B, a.T), 256); }

FwdK to_fwd(const lbwn_layer_args& a) {
  FwdK k;
  k.x_in = a.x_in; k.x_out = a.x_out; k.z = a.z; k.wpack = a.wpack; k.gc_tab = a.gc_tab; k.ids = a.ids;
  k.cond = a.cond; k.ldz = a.ldz; k.ldcond = a.ldcond; k.gc_ld = a.gc_ld ? a.gc_ld : 2L * a.Cd;
  k.B = a.B; k.T = a.T; k.H = a.H; k.d = a.d; k.Cr = a.Cr; k.Cd = a.Cd;
  return k;
}
BwdK to_bwd(const lbwn_layer_args& a) {
  BwdK k;
  k.x_in = a.x_in; k.wpack = a.wpack; k.dz_skip = a.dz_skip; k.g_a = a.g_a; k.g_c0 = a.g_c0;
  k.out_a = a.out_a; k.out_c0 = a.out_c0; k.slab = a.slab; k.gc_tab = a.gc_tab; k.ids = a.ids; k.cond = a.cond;
  k.dv_out = a.dv_out; k.gc_dtab = a.gc_dtab; k.lddz = a.lddz; k.ldcond = a.ldcond; k.lddv = a.lddv;
  k.gc_ld = a.gc_ld ? a.gc_ld : 2L * a.Cd;
  k.B = a.B; k.T = a.T; k.H = a.H; k.d = a.d; k.Cr = a.Cr; k.Cd = a.Cd; k.g_d = a.g_d; k.slab_stride = a.slab_stride;
  return k;
}

}  // namespace

int lbwn_layer_slab_stride() { return SLAB; }
int lbwn_layer_image_floats() { return WIMG; }

namespace {
// dL/d(halo buffer) of one layer from its backward's two outputs: out_a[t] = dL/dx[t] (own tap
// and residual) and out_c0[t] = dL/d(dilated tap input at t), which is halo row H + t - d.
__global__ void layer_dx_combine_kernel(const float* __restrict__ a, const float* __restrict__ c0, float* __restrict__ dx,
                                        int B, int T, int H, int d, int C) {
  const long total = (long)B * (H + T) * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const long br = e / C;
    const int row = (int)(br % (H + T)), b = (int)(br / (H + T));
    const int s = row - H;
    const long mb = (long)b * T;
    float v = 0.f;
    if (s >= 0) v = a[(mb + s) * C + c];
    if (s + d >= 0 && s + d < T) v += c0[(mb + s + d) * C + c];
    dx[e] = v;
  }
}
}  // namespace

int lbwn_layer_dx_combine_launch(const float* out_a, const float* out_c0, float* dx, int B, int T, int H, int d, int C,
                                 hipStream_t st) {
  const long total = (long)B * (H + T) * C;
  layer_dx_combine_kernel<<<(int)std::min<long>((total + 255) / 256, 4096), 256, 0, st>>>(out_a, out_c0, dx, B, T, H,
                                                                                          d, C);
  LBWN_CHECK_LAUNCH();
  return 0;
}
int lbwn_layer_image_x3_elems() { return XIMG_US; }
int lbwn_lc_image_x3_elems() { return LCIMG_US; }
int lbwn_lc_image16_elems() { return LC16IMG_US; }
int lbwn_chain_fwd_tile(int fwd_nw) { return fwd_nw ? 16 * fwd_nw : LP; }
int lbwn_lc_in_chain_ok(int Lo) { return Lo > 16 * (LC_K - 1) && Lo <= LC_KP && Lo % 4 == 0; }
int lbwn_layer_image_bx3_floats() { return BIMG_F; }
int lbwn_pack_layers_bx3_launch(const float* sig, const float* gate, const float* res, float* out, int L, int Cr,
                                int Cd, hipStream_t st) {
  LBWN_REQUIRE(Cr <= 32 && Cd <= 32 && (((uintptr_t)out) & 15) == 0, "pack_layers_bx3: bad arguments");
  pack_layers_bx3_kernel<<<L, 256, 0, st>>>(sig, gate, res, out, Cr, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_pack_layers_fb_x3_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                  const float* res, const float* res_b, unsigned short* fout, float* bout, int L,
                                  int Cr, int Cd, const float* skip_b, int Cs, float* bsum, const float* lc_sig,
                                  const float* lc_gate, int Lo, unsigned short* lcout, hipStream_t st, int lc16) {
  LBWN_REQUIRE(Cr <= 32 && Cd <= 32 && (((uintptr_t)fout) & 15) == 0 && (((uintptr_t)bout) & 15) == 0,
               "pack_layers_fb_x3: bad arguments");
  LBWN_REQUIRE(!lcout || (lc_sig && lc_gate && Lo >= 1 && Lo <= LC_KP && (((uintptr_t)lcout) & 15) == 0),
               "pack_layers_fb_x3: bad LC image arguments");
  const int nsum = (skip_b && bsum) ? (Cs + 255) / 256 : 0;
  const int nlc = lcout ? L : 0;
  pack_layers_fb_x3_kernel<<<2 * L + nlc + nsum, 256, 0, st>>>(sig, gate, sig_b, gate_b, res, res_b, fout, bout, L, Cr,
                                                               Cd, skip_b, Cs, bsum, lc_sig, lc_gate, Lo, lcout,
                                                               lc16);
  LBWN_CHECK_LAUNCH();
  return 0;
}
int lbwn_step_prologue_launch(const lbwn_prologue_args& a, hipStream_t st) {
  LBWN_REQUIRE(a.Cr <= 32 && a.Cd <= 32 && (((uintptr_t)a.fout) & 15) == 0 && (((uintptr_t)a.bout) & 15) == 0,
               "step_prologue: bad pack arguments");
  LBWN_REQUIRE(!a.lcout || (a.lc_sig && a.lc_gate && a.Lo >= 1 && a.Lo <= LC_KP && (((uintptr_t)a.lcout) & 15) == 0),
               "step_prologue: bad LC image arguments");
  LBWN_REQUIRE(a.njobs >= 0 && a.njobs <= 6 && a.zero_bytes % 4 == 0 && a.q && a.pre && a.X && a.save,
               "step_prologue: bad arguments");
  PrologueK k;
  memset(&k, 0, sizeof(k));
  k.a = a;
  long most = 0;
  for (int j = 0; j < a.njobs; ++j) {
    LBWN_REQUIRE(a.W[j] && a.out[j] && a.rows[j] > 0 && a.K[j] > 0, "step_prologue: bad split job");
    k.jb.W[j] = a.W[j]; k.jb.ldw[j] = a.ldw[j]; k.jb.rows[j] = a.rows[j]; k.jb.K[j] = a.K[j];
    k.jb.trans[j] = a.trans[j]; k.jb.out[j] = a.out[j];
    most = std::max(most, (long)a.rows[j] * ((a.K[j] + PLANE_BK - 1) / PLANE_BK) * (PLANE_BK / 2));
  }
  auto blocks = [](long n, long per, long cap) { return (int)std::max(1L, std::min(cap, (n + per - 1) / per)); };
  k.ns = blocks(most, 1024, 256);                                        // 4 pairs per thread
  LBWN_REQUIRE((long)a.B * a.T * a.Cr < (1L << 31) && (long)dsep_rows(a.L, a.nbl, 1) * a.B * a.Cr < (1L << 31),
               "step_prologue: x / SAVE exceed 32-bit indexing");
  k.ev4 = embed_v4(a.pre, a.pre_b, a.X, a.Cr);
  k.dv4 = dsep_v4(a.X, a.xls, a.save, a.Cr);
  k.ne = blocks((long)a.B * a.T * (k.ev4 ? a.Cr / 4 : a.Cr), 256, 2048);   // one item per thread
  k.nd = blocks((long)dsep_rows(a.L, a.nbl, a.B) * (k.dv4 ? a.Cr / 4 : a.Cr), 256, 2048);
  k.nz = a.zero_bytes ? blocks((long)(a.zero_bytes / 4), 1024, 256) : 0;
  k.np = 2 * a.L + (a.lcout ? a.L : 0) + ((a.skip_b && a.bsum) ? (a.Cs + 255) / 256 : 0);
  const long grid = (long)k.ns * a.njobs + k.ne + k.nd + k.nz + k.np;
  step_prologue_kernel<<<(unsigned)grid, 256, 0, st>>>(k);
  LBWN_CHECK_LAUNCH();
  return 0;
}
int lbwn_pack_layers_x3_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                               const float* res, const float* res_b, unsigned short* out, int L, int Cr, int Cd,
                               hipStream_t st) {
  LBWN_REQUIRE(Cr <= 32 && Cd <= 32 && (((uintptr_t)out) & 15) == 0, "pack_layers_x3: bad arguments");
  pack_layers_x3_kernel<<<L, 256, 0, st>>>(sig, gate, sig_b, gate_b, res, res_b, out, Cr, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}
int lbwn_layer_nblocks(int B, int T) { return B * ((T + LP - 1) / LP); }
int lbwn_layer_bwd_grid(int B, int T) { return std::min(lbwn_layer_nblocks(B, T), 256); }

int lbwn_pack_layers_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                            const float* res, const float* res_b, float* out, int L, int Cr, int Cd, hipStream_t st) {
  pack_layers_kernel<<<L, 256, 0, st>>>(sig, gate, sig_b, gate_b, res, res_b, out, Cr, Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

static int check_layer(const lbwn_layer_args& a) {
  LBWN_REQUIRE(a.Cr >= 1 && a.Cr <= 32 && a.Cd >= 1 && a.Cd <= 32, "layer: n_res/n_dil must be in [1,32]");
  LBWN_REQUIRE(a.d >= 1 && a.d <= a.H, "layer: dilation %d exceeds halo %d", a.d, a.H);
  LBWN_REQUIRE(a.B >= 1 && a.T >= 1, "layer: empty batch");
  LBWN_REQUIRE(a.wpack && (((uintptr_t)a.wpack) & 15) == 0, "layer: packed weight image missing/misaligned");
  if (a.Cr == 32) LBWN_REQUIRE((((uintptr_t)a.x_in) & 15) == 0, "layer: x not 16-B aligned");
  return 0;
}

int lbwn_layer_fwd_launch(const lbwn_layer_args& a, hipStream_t st) {
  if (int e = check_layer(a)) return e;
  layer_fwd_kernel<<<grid_fwd(a), 256, 0, st>>>(to_fwd(a));
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_bwd_launch(const lbwn_layer_args& a, hipStream_t st) {
  if (int e = check_layer(a)) return e;
  LBWN_REQUIRE(a.slab && a.slab_stride >= SLAB, "layer bwd: slab missing");
  layer_bwd_kernel<<<grid_bwd(a), 256, 0, st>>>(to_bwd(a));
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_reduce_launch(const lbwn_layer_red_args& r, hipStream_t st) {
  LBWN_REQUIRE(r.slab && r.nparts >= 1 && r.stride >= SLAB, "layer reduce: bad slab");
  RedK k;
  k.slab = r.slab; k.dsig = r.dsig; k.dgate = r.dgate; k.dres = r.dres;
  k.dbsig = r.dbsig; k.dbgate = r.dbgate; k.dbres = r.dbres;
  k.nparts = r.nparts; k.stride = r.stride; k.Cr = r.Cr; k.Cd = r.Cd;
  layer_reduce_kernel<<<(SLAB + 31) / 32, 256, 0, st>>>(k);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_chain_fwd_lds_bytes() { return CF_LDS * 4; }

// the untraced or the traced instantiation of one forward chain
static void fwd_launch(bool traced, void (*plain)(ChainFK), void (*traced_k)(ChainFK), int grid, const ChainFK& k,
                       hipStream_t st) {
  if (traced) hipLaunchKernelGGL(traced_k, dim3(grid), dim3(256), 0, st, k);
  else hipLaunchKernelGGL(plain, dim3(grid), dim3(256), 0, st, k);
}

// the 16-position-wave forward chain of NW waves (64·NW threads), by LC / conditioning mode
template <int NW>
static void launch_fwd16(bool tr, bool lc, int cm, int grid, const ChainFK& k, hipStream_t st) {
  void (*f)(ChainFK);
  if (lc) f = cm == 0 ? (tr ? chain_fwd16_kernel<NW, true, 0, true> : chain_fwd16_kernel<NW, true, 0, false>)
                      : (tr ? chain_fwd16_kernel<NW, true, 1, true> : chain_fwd16_kernel<NW, true, 1, false>);
  else if (cm == 0) f = tr ? chain_fwd16_kernel<NW, false, 0, true> : chain_fwd16_kernel<NW, false, 0, false>;
  else if (cm == 1) f = tr ? chain_fwd16_kernel<NW, false, 1, true> : chain_fwd16_kernel<NW, false, 1, false>;
  else f = tr ? chain_fwd16_kernel<NW, false, 2, true> : chain_fwd16_kernel<NW, false, 2, false>;
  hipLaunchKernelGGL(f, dim3(grid), dim3(64 * NW), 0, st, k);
}

int lbwn_chain_fwd_launch(const lbwn_chain_args& c, hipStream_t st) {
  LBWN_REQUIRE(c.Cr == 32 && c.Cd == 32, "chain fwd: n_res = n_dil = 32 only");
  LBWN_REQUIRE(c.grid >= 1 && c.flags && c.status, "chain fwd: bad launch state");
  LBWN_REQUIRE((((uintptr_t)c.X) & 15) == 0 && (c.xls & 3) == 0, "chain fwd: x not 16-B aligned");
  ChainFK k;
  k.X = c.X; k.xls = c.xls; k.Z = c.Z; k.ldz = c.ldz; k.wpack = c.wpack;
  k.gc_tab = c.gc_tab; k.gc_ld = c.gc_ld; k.ids = c.ids; k.cond = c.cond; k.ldcond = c.ldcond;
  k.flags = c.flags; k.status = c.status;
  k.B = c.B; k.T = c.T; k.H = c.H; k.L = c.L; k.nbl = c.nbl; k.Cd = c.Cd;
  k.trace = c.trace; k.trace_blk = c.trace_blk;
  k.ximg = c.wpack_x3;
  k.xcd = c.xcd;
  k.SG = c.SG; k.sgls = c.sgls;
  k.lcact = c.lcact; k.lcimg = c.lcimg; k.Lo = c.Lo;
  LBWN_REQUIRE(!c.wpack_x3 || (((uintptr_t)c.wpack_x3) & 15) == 0, "chain fwd: split images not 16-B aligned");
  const bool lc = c.lcimg != nullptr;
  if (lc)
    LBWN_REQUIRE(c.wpack_x3 && c.lcact && !c.cond && c.Lo > 16 * (LC_K - 1) && c.Lo <= LC_KP && c.Lo % 4 == 0 &&
                     (((uintptr_t)c.lcact) & 15) == 0 && (((uintptr_t)c.lcimg) & 15) == 0,
                 "chain fwd: in-chain LC needs the split images, %d < n_lc_out <= %d, aligned rows", 16 * (LC_K - 1),
                 LC_KP);
  LBWN_REQUIRE(c.fwd_nw == 0 || ((c.fwd_nw == 4 || c.fwd_nw == 8) && c.wpack_x3 && c.SG),
               "chain fwd: 16-position waves need the split images and the SG rows, 4 or 8 waves");
  const int tp = lbwn_chain_fwd_tile(c.fwd_nw);
  const int tps = (c.T + tp - 1) / tp;
  // hand-off flags only: the status word is sticky for the whole step
  if (!c.flags_zeroed) {
    if (int e = lbwn_zero_launch(c.flags, ((size_t)c.B * tps * 4 + 15) / 16 * 16, st)) return e;
  }
  const int cm = (!c.gc_tab && !c.cond) ? 0 : (c.gc_tab && !c.cond) ? 1 : 2;
  const bool tr = c.trace != nullptr;
  if (c.fwd_nw == 8) launch_fwd16<8>(tr, lc, cm, c.grid, k, st);
  else if (c.fwd_nw == 4) launch_fwd16<4>(tr, lc, cm, c.grid, k, st);
  else if (lc) {
    if (cm == 0) fwd_launch(c.trace != nullptr, chain_fwd_kernel<true, true, 0, false>, chain_fwd_kernel<true, true, 0, true>, c.grid, k, st);
    else fwd_launch(c.trace != nullptr, chain_fwd_kernel<true, true, 1, false>, chain_fwd_kernel<true, true, 1, true>, c.grid, k, st);   // lc: cond is null
  } else if (c.wpack_x3) {
    if (cm == 0) fwd_launch(c.trace != nullptr, chain_fwd_kernel<true, false, 0, false>, chain_fwd_kernel<true, false, 0, true>, c.grid, k, st);
    else if (cm == 1) fwd_launch(c.trace != nullptr, chain_fwd_kernel<true, false, 1, false>, chain_fwd_kernel<true, false, 1, true>, c.grid, k, st);
    else fwd_launch(c.trace != nullptr, chain_fwd_kernel<true, false, 2, false>, chain_fwd_kernel<true, false, 2, true>, c.grid, k, st);
  } else {
    if (cm == 0) fwd_launch(c.trace != nullptr, chain_fwd_kernel<false, false, 0, false>, chain_fwd_kernel<false, false, 0, true>, c.grid, k, st);
    else fwd_launch(c.trace != nullptr, chain_fwd_kernel<false, false, 2, false>, chain_fwd_kernel<false, false, 2, true>, c.grid, k, st);
  }
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_chain_bwd_launch(const lbwn_chain_args& c, hipStream_t st) {
  LBWN_REQUIRE(c.Cr == 32 && c.Cd == 32, "chain bwd: n_res = n_dil = 32 only");
  LBWN_REQUIRE(c.grid >= 1 && c.flags && c.status && c.slab && c.ocg && c.dx0_a && c.dx0_c && c.DZ,
               "chain bwd: bad launch state");
  ChainBK k;
  k.X = c.X; k.xls = c.xls; k.DZ = c.DZ; k.lddz = c.ldz; k.dzls = c.dzls; k.wpack = c.wpack; k.slab = c.slab;
  k.ocg = c.ocg; k.ocls = c.ocls; k.dx0_a = c.dx0_a; k.dx0_c = c.dx0_c;
  k.gc_tab = c.gc_tab; k.gc_ld = c.gc_ld; k.ids = c.ids; k.cond = c.cond; k.ldcond = c.ldcond;
  k.dv_out = c.dv_out; k.lddv = c.lddv; k.gc_dtab = c.gc_dtab; k.tile_gid = c.tile_gid;
  k.dvks = c.dvks;
  k.flags = c.flags; k.status = c.status;
  k.B = c.B; k.T = c.T; k.H = c.H; k.L = c.L; k.nbl = c.nbl; k.Cd = c.Cd;
  k.trace = c.trace ? c.trace + 16L * c.L : nullptr; k.trace_blk = c.trace_blk;
  k.xcd = c.xcd;
  k.Zf = c.Z; k.SG = c.SG; k.sgls = c.sgls; k.bimg = c.bimg;
  const bool x3 = c.bimg && c.SG && c.Z;
  if (x3) LBWN_REQUIRE((((uintptr_t)c.bimg) & 15) == 0 && (((uintptr_t)c.SG) & 15) == 0 && (c.ldz & 3) == 0,
                       "chain bwd x3: misaligned images / rows");
  LBWN_REQUIRE(c.bwd_nw == 0 || ((c.bwd_nw == 4 || c.bwd_nw == 8) && x3),
               "chain bwd: 16-position waves need the bf16-split form, 4 or 8 waves");
  const int tp = lbwn_chain_fwd_tile(c.bwd_nw);
  const int tps = (c.T + tp - 1) / tp;
  // hand-off flags only: the status word is sticky for the whole step
  if (!c.flags_zeroed) {
    if (int e = lbwn_zero_launch(c.flags, ((size_t)c.B * tps * 4 + 15) / 16 * 16, st)) return e;
  }
  LBWN_REQUIRE(x3 == (c.dzls > 0), "chain bwd: the bf16-split chain reads dZ in chain order (dzls), the f32 chain in rows");
  if (c.bwd_nw)   // 32-bit byte offsets of the per-lane row loads (chain_bwd16_kernel load_regs)
    LBWN_REQUIRE(c.dzls * 4 < 0x7fffffffL && c.sgls * 4 < 0x7fffffffL && (long)c.B * c.T * c.ldz * 4 < 0x7fffffffL,
                 "chain bwd: dZ / SG layer or z rows past 2 GiB");
  k.gx = c.gx; k.gxls = c.gxls;
  if (c.gx)   // weight gradients outside the chain (layer_wgrad_kernel): DV and G exported
    LBWN_REQUIRE(c.bwd_nw == 8 && c.dv_out && c.dvks > 0 && c.gxls >= (long)c.B * c.T * 32,
                 "chain bwd: the export form needs 8 waves and the k-blocked DV export");
  if (c.bwd_nw == 8) {
    if (c.gx) {
      if (k.trace) chain_bwd16_kernel<8, true, false><<<c.grid, 512, 0, st>>>(k);
      else chain_bwd16_kernel<8, false, false><<<c.grid, 512, 0, st>>>(k);
    } else if (k.trace) chain_bwd16_kernel<8, true, true><<<c.grid, 512, 0, st>>>(k);
    else chain_bwd16_kernel<8, false, true><<<c.grid, 512, 0, st>>>(k);
  } else if (c.bwd_nw == 4) {
    if (k.trace) chain_bwd16_kernel<4, true, true><<<c.grid, 256, 0, st>>>(k);
    else chain_bwd16_kernel<4, false, true><<<c.grid, 256, 0, st>>>(k);
  } else if (x3 && k.trace) chain_bwd_x3_kernel<true><<<c.grid, 256, 0, st>>>(k);
  else if (x3) chain_bwd_x3_kernel<false><<<c.grid, 256, 0, st>>>(k);
  else chain_bwd_kernel<<<c.grid, 256, 0, st>>>(k);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_reduce_all_launch(const lbwn_layer_red_args& r, int L, long slab_layer, hipStream_t st) {
  LBWN_REQUIRE(r.slab && r.nparts >= 1 && r.stride >= SLAB && L >= 1, "layer reduce: bad slab");
  RedK k;
  k.slab = r.slab; k.dsig = r.dsig; k.dgate = r.dgate; k.dres = r.dres;
  k.dbsig = r.dbsig; k.dbgate = r.dbgate; k.dbres = r.dbres;
  k.nparts = r.nparts; k.stride = r.stride; k.Cr = r.Cr; k.Cd = r.Cd;
  layer_reduce_all_kernel<<<dim3((SLAB + 31) / 32, L), 256, 0, st>>>(k, slab_layer, 2L * r.Cr * r.Cd,
                                                                    (long)r.Cd * r.Cr, r.Cd);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_slab_floats() { return SLAB; }

namespace {
// gtab[id][l·64 + c] += Σ over tiles with tile_gid == id (in tile order) of the tile's dv column
// sums slab[l][tile][5120 + c].  Block = (layer, id), thread = column: the block scans the tile ids
// 64 at a time (one per lane, ballot), then adds its matching tiles' partials in tile order
// (deterministic; blocks of ids with no uniform tile only scan).  Side stream beside dSKIP, where
// every dependent round trip is long: few VGPRs, 1,024 tile ids loaded at once (16 per lane) and
// the matching tiles listed in LDS in tile order, then their partials loaded 16 at a time (a
// ballot and a batch of 4 loads per 64 tiles ran 117 us at C4, one load per tile 154 us).
constexpr int GTS_CHUNK = 1024;
__global__ __launch_bounds__(64) void gc_tile_sum_kernel(const float* __restrict__ slab, long slab_layer, long tstride,
                                                         int ntiles, const int* __restrict__ tile_gid, float* gtab,
                                                         long ld) {
  __shared__ int lst[GTS_CHUNK];
  const int l = blockIdx.x, id = blockIdx.y, c = threadIdx.x;
  // the layer's partials through a buffer resource: a load's tile offset is one SGPR (the list
  // entry is wave-uniform), so a batch of 16 costs 16 VGPRs, not 16 64-bit addresses
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(slab + l * slab_layer), (short)0, (int)min(slab_layer * 4, 0x7fffffffL), BUF_DW3);
  const __amdgpu_buffer_rsrc_t rg =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(tile_gid), (short)0, ntiles * 4, BUF_DW3);
  float acc = 0.f;
  bool any = false;
  for (int s0 = 0; s0 < ntiles; s0 += GTS_CHUNK) {
    int gid[GTS_CHUNK / 64];
#pragma unroll
    for (int k = 0; k < GTS_CHUNK / 64; ++k)   // past the end: 0 from the range-checked buffer offset, masked below
      gid[k] = (int)__builtin_amdgcn_raw_buffer_load_b32(rg, (s0 + c) * 4 + 256 * k, 0, 0);
    int n = 0;
#pragma unroll
    for (int k = 0; k < GTS_CHUNK / 64; ++k) {
      const int t = s0 + 64 * k + c;
      const bool hit = t < ntiles && gid[k] == id;
      const unsigned long long m = __ballot(hit);
      if (hit) lst[n + __popcll(m & ((1ull << c) - 1ull))] = t;
      n += __popcll(m);
    }
    any |= n > 0;
    __syncthreads();
    for (int i = 0; i < n; i += 16) {   // in tile order
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rs, c * 4, __builtin_amdgcn_readfirstlane(lst[min(i + k, n - 1)]) * (int)tstride * 4, 0));
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (i + k < n) acc += v[k];
    }
    __syncthreads();   // the list is rewritten by the next chunk
  }
  if (any) gtab[(long)id * ld + (long)l * 64 + c] += acc;
}
}  // namespace

int lbwn_gc_tile_sum_launch(const float* slab, int L, int ntiles, const int* tile_gid, float* gtab, long ld,
                            int ncat1, hipStream_t st) {
  LBWN_REQUIRE(ncat1 >= 1 && slab && tile_gid && gtab, "gc tile sums: bad arguments");
  gc_tile_sum_kernel<<<dim3(L, ncat1), 64, 0, st>>>(slab + 5120, (long)ntiles * SLAB, SLAB, ntiles, tile_gid, gtab, ld);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_wgrad_tiles_per_chunk(int ntiles, int L, int ncu) {
  // about eight blocks of the grid per CU (two resident per CU): long per-wave streams, a small
  // slab ([L][nchunk][SLAB]: 33 MB at C2 and C4)
  int tpc = 8;
  while (tpc < WG_TPC_MAX && (long)(ntiles / (2 * tpc)) * L >= 8L * ncu) tpc *= 2;
  return tpc;
}

int lbwn_layer_wgrad_launch(const lbwn_wgrad_args& g, hipStream_t st) {
  LBWN_REQUIRE(g.X && g.Z && g.DV && g.GX && g.slab && g.tpc >= 1 && g.tpc <= WG_TPC_MAX && g.stride >= SLAB,
               "layer wgrad: bad arguments");
  LBWN_REQUIRE(!g.gcs || (g.ids && g.tile_gid && g.gtab), "layer wgrad: GC needs ids, tile ids and the tables");
  const int tps = (g.T + 127) / 128, ntiles = g.B * tps;
  // 32-bit lane offsets (buffer loads): z rows, the exports, x
  LBWN_REQUIRE((long)g.B * g.T * g.lddz * 4 < 0x7fffffffL && g.dvks * 4 < 0x7fffffffL && g.gxls * 4 < 0x7fffffffL &&
                   g.xls * 4 < 0x7fffffffL && g.dvks >= (long)g.B * g.T * 32 && g.gxls >= (long)g.B * g.T * 32,
               "layer wgrad: rows past 2 GiB per layer");
  WgK k;
  k.X = g.X; k.xls = g.xls; k.Z = g.Z; k.lddz = g.lddz; k.DV = g.DV; k.dvks = g.dvks; k.GX = g.GX; k.gxls = g.gxls;
  k.slab = g.slab; k.stride = g.stride;
  k.ids = g.ids; k.tile_gid = g.tile_gid; k.gcs = g.gcs; k.gtab = g.gtab; k.gc_ld = g.gc_ld;
  k.B = g.B; k.T = g.T; k.H = g.H; k.L = g.L; k.nbl = g.nbl; k.tps = tps; k.ntiles = ntiles; k.tpc = g.tpc;
  k.nchunk = (ntiles + g.tpc - 1) / g.tpc;
  const dim3 grid(k.nchunk, g.L);
  if (g.gcs) layer_wgrad_kernel<true><<<grid, 256, 0, st>>>(k);
  else layer_wgrad_kernel<false><<<grid, 256, 0, st>>>(k);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_gc_tile_sum_rows_launch(const float* gcs, int L, int ntiles, const int* tile_gid, float* gtab, long ld,
                                 int ncat1, hipStream_t st) {
  LBWN_REQUIRE(ncat1 >= 1 && gcs && tile_gid && gtab, "gc tile sums: bad arguments");
  gc_tile_sum_kernel<<<dim3(L, ncat1), 64, 0, st>>>(gcs, (long)ntiles * 64, 64, ntiles, tile_gid, gtab, ld);
  LBWN_CHECK_LAUNCH();
  return 0;
}
