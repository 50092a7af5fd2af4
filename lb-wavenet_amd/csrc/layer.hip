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
#include "common.h"
#include "kernels.h"

namespace {

constexpr int LP = LBWN_LAYER_POS;  // positions per tile (4 waves × 32)
constexpr int XS = 36;              // padded LDS row for 32-channel tiles (b128 conflict-free)
constexpr int WS = 68;              // padded row of the [64 in][64 out] conv weight image
constexpr int DS = 68;              // dv tile row [pos][64]
constexpr int WIMG = 64 * WS + 32 * XS + 96;  // packed per-layer image (floats), multiple of 4
constexpr int SLAB = 2048 + 2048 + 1024 + 96;
constexpr int RED_PARTS = 32;       // deferred reduction: parts prefetched per thread (8 lanes × 32)
// Timing-only ablation switches (tools/ablate.sh); 0 in every real build.
#ifndef LBWN_ABL
#define LBWN_ABL 0
#endif

// Compact kernel arguments (the full lbwn_layer_args by value spilled ~100 SGPRs).
struct FwdK {
  const float* x_in; float* x_out; float* z; const float* wpack;
  const float* gc_tab; const int* ids; const float* cond;
  long ldz, ldcond;
  int B, T, H, d, Cr, Cd;
};
struct BwdK {
  const float* x_in; const float* wpack; const float* dz_skip;
  const float* g_a; const float* g_c0; float* out_a; float* out_c0; float* slab;
  const float* gc_tab; const int* ids; const float* cond; float* dv_out; float* gc_dtab;
  long lddz, ldcond, lddv;
  int B, T, H, d, Cr, Cd, g_d, slab_stride;
  // deferred reduction
  const float* red_slab; float* red_dsig; float* red_dgate; float* red_dres;
  float* red_dbsig; float* red_dbgate; float* red_dbres;
  int red_nparts, red_stride;
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

// ---- LDS staging ---------------------------------------------------------------------

// dst[r][0..31] = x row (t0 + r + shift) of the halo buffer xb, zero if t0+r >= T.
LBWN_DEV void stage_rows(float* dst, const float* __restrict__ xb, int t0, int shift, int T, int H, int C,
                         int tid) {
  if (C == 32) {
    floatx4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      const int r = e >> 3, c4 = (e & 7) * 4;
      v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (t0 + r < T) v[i] = *(const floatx4*)(xb + (long)(H + t0 + r + shift) * 32 + c4);
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
      v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      u[i] = v[i];
      if (t < T) v[i] = *(const floatx4*)(ga + (mb + t) * 32 + c4);
      if (t + gd < T) u[i] = *(const floatx4*)(gc + (mb + t + gd) * 32 + c4);
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
        if (t + gd < T) v += gc[(mb + t + gd) * C + c];
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
    const float* cs = a.gc_tab ? a.gc_tab + (long)a.ids[m] * 2 * a.Cd : nullptr;
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

// ---- deferred slab reduction -------------------------------------------------------------

// Destination of slab column c (padded 32-channel layout) in reference layout.
LBWN_DEV void slab_store(const BwdK& a, int c, float tot) {
  const int Cr = a.Cr, Cd = a.Cd;
  if (c < 4096) {
    const int cc = c & 2047, tap = cc >> 10, in = (cc >> 5) & 31, o = cc & 31;
    float* dst = c < 2048 ? a.red_dsig : a.red_dgate;
    if (in < Cr && o < Cd) dst[(tap * Cr + in) * Cd + o] = tot;
  } else if (c < 5120) {
    const int cc = c - 4096, zc = cc >> 5, o = cc & 31;
    if (zc < Cd && o < Cr) a.red_dres[zc * Cr + o] = tot;
  } else {
    const int cc = c - 5120, seg = cc >> 5, o = cc & 31;
    if (seg == 0 && a.red_dbsig && o < Cd) a.red_dbsig[o] = tot;
    if (seg == 1 && a.red_dbgate && o < Cd) a.red_dbgate[o] = tot;
    if (seg == 2 && a.red_dbres && o < Cr) a.red_dbres[o] = tot;
  }
}

// Column group `grp` (32 columns) summed over all parts: thread = (part lane p8, column);
// `pre` holds parts p8, p8+8, ... (up to RED_PARTS) loaded earlier.
LBWN_DEV void slab_group_finish(const BwdK& a, int grp, const float (&pre)[RED_PARTS], float* scratch,
                                int tid) {
  const int c = grp * 32 + (tid & 31), p8 = tid >> 5;
  float s = 0.f;
  if (c < SLAB) {
#pragma unroll
    for (int j = 0; j < RED_PARTS; ++j) s += pre[j];
    for (int p = p8 + 8 * RED_PARTS; p < a.red_nparts; p += 8) s += a.red_slab[(long)p * a.red_stride + c];
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

LBWN_DEV void slab_group_prefetch(const BwdK& a, int grp, float (&pre)[RED_PARTS], int tid) {
  const int c = grp * 32 + (tid & 31), p8 = tid >> 5;
#pragma unroll
  for (int j = 0; j < RED_PARTS; ++j) {
    const int p = p8 + 8 * j;
    pre[j] = (c < SLAB && p < a.red_nparts) ? a.red_slab[(long)p * a.red_stride + c] : 0.f;
  }
}

// ---- backward ----------------------------------------------------------------------------

__global__ __launch_bounds__(256) void layer_bwd_kernel(BwdK a) {
  __shared__ __attribute__((aligned(16))) float sm[3 * LP * XS + WIMG + LP * DS + LP * XS + 4 * 1024];
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* G = Xc + LP * XS;
  float* Ws = G + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* DV = bs + 96;               // [LP][DS]   dv (sig | gate), position-major
  float* ZT = DV + LP * DS;          // [LP][XS]   z, position-major
  float* RED = ZT + LP * XS;         // 4 × 1024
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;
  const int tps = (a.T + LP - 1) / LP, ntiles = a.B * tps;
  const int ngroups = (SLAB + 31) / 32;

  // deferred reduction of the deeper layer's partials: issue the loads now, sum at the end
  float pre[RED_PARTS];
  const bool red = !(LBWN_ABL & 1) && a.red_slab && (int)blockIdx.x < ngroups;
  if (red) slab_group_prefetch(a, blockIdx.x, pre, tid);

  stage_image(Ws, a.wpack, tid);
  floatx16 accW, accR;  // tile w of dSIG/dGATE (w: 0 sig·prev, 1 sig·cur, 2 gate·prev, 3 gate·cur), dRES part
#pragma unroll
  for (int r = 0; r < 16; ++r) { accW[r] = 0.f; accR[r] = 0.f; }
  float bsum = 0.f;  // bias partial: tid<64 dv column, 64..95 g column

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, t0 = (tile % tps) * LP;
    const long mb = (long)b * a.T;
    const float* xb = a.x_in + (long)b * (a.H + a.T) * a.Cr;
    if (tile != (int)blockIdx.x) __syncthreads();
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
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        if (valid) v = *(const floatx4*)(a.dz_skip + m * a.lddz + 8 * q + 4 * h);
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
    // 3. dvᵀ, parked position-major with z for the weight-grad products
    floatx16 dvs, dvg, z;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      z[r] = th[r] * sg[r];
      dvs[r] = dz[r] * sg[r] * (1.f - th[r] * th[r]);
      dvg[r] = dz[r] * th[r] * sg[r] * (1.f - sg[r]);
    }
    float* dvrow = DV + (32 * w + pi) * DS;
    float* zrow = ZT + (32 * w + pi) * XS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *(floatx4*)(dvrow + 8 * q + 4 * h) = floatx4{dvs[4 * q], dvs[4 * q + 1], dvs[4 * q + 2], dvs[4 * q + 3]};
      *(floatx4*)(dvrow + 32 + 8 * q + 4 * h) = floatx4{dvg[4 * q], dvg[4 * q + 1], dvg[4 * q + 2], dvg[4 * q + 3]};
      *(floatx4*)(zrow + 8 * q + 4 * h) = floatx4{z[4 * q], z[4 * q + 1], z[4 * q + 2], z[4 * q + 3]};
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
    __syncthreads();  // DV / ZT of every wave visible

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
    if (a.gc_dtab) {
      const int tw0 = t0 + 32 * w;
      const int nv = min(32, a.T - tw0);
      if (nv > 0) {
        const int* idw = a.ids + mb + tw0;
        const int id0 = idw[0];
        bool uni = true;
        for (int p = 1; p < nv; ++p) uni &= (idw[p] == id0);
        const int o = lane, oc = o & 31;
        const float* dvw = DV + 32 * w * DS;
        if (oc < a.Cd) {
          const int col = o < 32 ? oc : a.Cd + oc;
          if (uni) {
            float s = 0.f;
            for (int p = 0; p < nv; ++p) s += dvw[p * DS + o];
            atomicAdd(a.gc_dtab + (long)id0 * 2 * a.Cd + col, s);
          } else {
            for (int p = 0; p < nv; ++p) atomicAdd(a.gc_dtab + (long)idw[p] * 2 * a.Cd + col, dvw[p * DS + o]);
          }
        }
      }
    }
  }

  // 8. block partial -> slab: tiles 0..3 straight from their wave, dRES summed over waves
  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    slab[w * 1024 + acc_row(r, h) * 32 + pi] = accW[r];
    RED[w * 1024 + acc_row(r, h) * 32 + pi] = accR[r];
  }
  __syncthreads();
  for (int e = tid; e < 1024; e += 256) slab[4096 + e] = ((RED[e] + RED[1024 + e]) + RED[2048 + e]) + RED[3072 + e];
  if (tid < 96) slab[5120 + tid] = bsum;
  // 9. finish the deferred reduction (remaining groups when the grid is small)
  if (red) slab_group_finish(a, blockIdx.x, pre, RED, tid);
  if (!(LBWN_ABL & 1) && a.red_slab) {
    float none[RED_PARTS];
    for (int grp = blockIdx.x + gridDim.x; grp < ngroups; grp += gridDim.x) {
      slab_group_prefetch(a, grp, none, tid);
      slab_group_finish(a, grp, none, RED, tid);
    }
  }
}

__global__ __launch_bounds__(256) void layer_reduce_kernel(BwdK a) {
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
  k.cond = a.cond; k.ldz = a.ldz; k.ldcond = a.ldcond;
  k.B = a.B; k.T = a.T; k.H = a.H; k.d = a.d; k.Cr = a.Cr; k.Cd = a.Cd;
  return k;
}
BwdK to_bwd(const lbwn_layer_args& a) {
  BwdK k;
  k.x_in = a.x_in; k.wpack = a.wpack; k.dz_skip = a.dz_skip; k.g_a = a.g_a; k.g_c0 = a.g_c0;
  k.out_a = a.out_a; k.out_c0 = a.out_c0; k.slab = a.slab; k.gc_tab = a.gc_tab; k.ids = a.ids; k.cond = a.cond;
  k.dv_out = a.dv_out; k.gc_dtab = a.gc_dtab; k.lddz = a.lddz; k.ldcond = a.ldcond; k.lddv = a.lddv;
  k.B = a.B; k.T = a.T; k.H = a.H; k.d = a.d; k.Cr = a.Cr; k.Cd = a.Cd; k.g_d = a.g_d; k.slab_stride = a.slab_stride;
  k.red_slab = a.red_slab; k.red_dsig = a.red_dsig; k.red_dgate = a.red_dgate; k.red_dres = a.red_dres;
  k.red_dbsig = a.red_dbsig; k.red_dbgate = a.red_dbgate; k.red_dbres = a.red_dbres;
  k.red_nparts = a.red_nparts; k.red_stride = a.red_stride;
  return k;
}

}  // namespace

int lbwn_layer_slab_stride() { return SLAB; }
int lbwn_layer_image_floats() { return WIMG; }
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
  LBWN_REQUIRE(!a.red_slab || a.red_nparts <= 8 * RED_PARTS || true, "unreachable");
  layer_bwd_kernel<<<grid_bwd(a), 256, 0, st>>>(to_bwd(a));
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_reduce_launch(const lbwn_layer_args& a, hipStream_t st) {
  layer_reduce_kernel<<<(SLAB + 31) / 32, 256, 0, st>>>(to_bwd(a));
  LBWN_CHECK_LAUNCH();
  return 0;
}
