// One WaveNet residual layer, forward and backward (tmodel.py:117-184, :313-325).
//
// Layout: activations are channels-last rows; x_l lives in a per-stream buffer
// [B][H+T][Cr] whose first H rows are a halo: rows [H-d, H) hold SAVE_l, so the dilated
// tap x[t-d] (or SAVE for t<d, tmodel.py:122-127) is simply row H+t-d.  A block owns 128
// consecutive positions of one stream; both taps are staged into LDS with coalesced
// 16-B loads (Xp = rows t-d, Xc = rows t), then each wave computes a 32-position tile with
// v_mfma_f32_32x32x2_f32 in the TRANSPOSED orientation (channels on MFMA rows, positions on
// lanes) so that the gate output z is already the B operand of the residual/weight-grad
// products (no lane shuffles):
//   vᵀ[64 × 32pos] = Wcatᵀ[64 out × 64 in] · [x[t-d] | x[t]]ᵀ   (sig rows 0-31, gate 32-63)
//   zᵀ = tanh(v_sig)·σ(v_gate);  x_{l+1}ᵀ = x_lᵀ + RESᵀ·zᵀ + b_res
// Channel counts up to 32 are supported (zero-padded in LDS); 32 takes the vector path.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int LP = LBWN_LAYER_POS;  // positions per block (4 waves × 32)
constexpr int XS = 36;              // padded LDS row for 32-channel tiles (b128 conflict-free)
constexpr int WS = 68;              // padded LDS row of the [64 in][64 out] conv weight image
constexpr int DS = 68;              // per-wave dv tile row [32 pos][64]
constexpr int SLAB = 2048 + 2048 + 1024 + 96;

// ---- LDS staging ---------------------------------------------------------------------

// rows r in [0,LP): dst[r][0..31] = src row (t0 + r + shift) of stream b, zero if outside [0,T)
// (shift < 0 reads into the halo, which is always inside the buffer).
LBWN_DEV void stage_rows(float* dst, const float* __restrict__ xb, int t0, int shift, int T, int H, int C,
                         int tid) {
  if (C == 32) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;  // 0..1023 float4 slots
      const int r = e >> 3, c4 = (e & 7) * 4;
      const int t = t0 + r;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (t < T) v = *(const floatx4*)(xb + (long)(H + t + shift) * 32 + c4);
      *(floatx4*)(dst + r * XS + c4) = v;
    }
  } else {
    for (int e = tid; e < LP * 32; e += 256) {
      const int r = e >> 5, c = e & 31;
      const int t = t0 + r;
      float v = 0.f;
      if (t < T && c < C) v = xb[(long)(H + t + shift) * C + c];
      dst[r * XS + c] = v;
    }
  }
}

// Plain [M][C] rows (no halo): dst[r] = src[(b*T + t0 + r + shift)], zero outside [0,T).
LBWN_DEV void stage_plain(float* dst, const float* __restrict__ src, long ld, int b, int t0, int shift, int T,
                          int C, int tid, bool add) {
  for (int e = tid; e < LP * 32; e += 256) {
    const int r = e >> 5, c = e & 31;
    const int t = t0 + r + shift;
    float v = 0.f;
    if (t0 + r < T && t < T && c < C) v = src[((long)b * T + t) * ld + c];
    if (add) dst[r * XS + c] += v;
    else dst[r * XS + c] = v;
  }
}

// conv weights -> Ws[k = tap*32 + in][out (sig 0..31 | gate 32..63)], RES -> Rs[c][o]
LBWN_DEV void stage_weights(float* Ws, float* Rs, float* bs, float* br, const lbwn_layer_args& a, int tid) {
  const int Cr = a.Cr, Cd = a.Cd;
  for (int e = tid; e < 64 * 64; e += 256) {
    const int k = e >> 6, o = e & 63;
    const int tap = k >> 5, in = k & 31, oc = o & 31;
    const float* W = (o < 32) ? a.w_sig : a.w_gate;
    float v = 0.f;
    if (in < Cr && oc < Cd) v = W[(tap * Cr + in) * Cd + oc];
    Ws[k * WS + o] = v;
  }
  for (int e = tid; e < 32 * 32; e += 256) {
    const int c = e >> 5, o = e & 31;
    Rs[c * XS + o] = (c < Cd && o < Cr) ? a.w_res[c * Cr + o] : 0.f;
  }
  if (tid < 64) {
    const int oc = tid & 31;
    const float* bb = tid < 32 ? a.b_sig : a.b_gate;
    bs[tid] = (bb && oc < Cd) ? bb[oc] : 0.f;
  } else if (tid < 96) {
    const int o = tid - 64;
    br[o] = (a.b_res && o < Cr) ? a.b_res[o] : 0.f;
  }
}

// vᵀ for this wave's 32 positions: acc_s/acc_g rows = out channel, lanes = position.
LBWN_DEV void conv_tile(const float* Xp, const float* Xc, const float* Ws, const float* bs,
                        const lbwn_layer_args& a, int b, int t, bool valid, int w, int lane, floatx16& acc_s,
                        floatx16& acc_g) {
  const int pi = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc_s[r] = bs[acc_row(r, h)];
    acc_g[r] = bs[32 + acc_row(r, h)];
  }
  if (valid && (a.gc_tab || a.cond)) {
    const long m = (long)b * a.T + t;
    const float* cs = a.gc_tab ? a.gc_tab + (long)a.ids[m] * 2 * a.Cd : a.cond + m * a.ldcond;
    if (a.gc_tab && a.cond) {
      // both: GC table row + LC projection row
      const float* cl = a.cond + m * a.ldcond;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = acc_row(r, h);
        if (o < a.Cd) {
          acc_s[r] += cs[o] + cl[o];
          acc_g[r] += cs[a.Cd + o] + cl[a.Cd + o];
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = acc_row(r, h);
        if (o < a.Cd) {
          acc_s[r] += cs[o];
          acc_g[r] += cs[a.Cd + o];
        }
      }
    }
  }
  const float* xp = Xp + (32 * w + pi) * XS;
  const float* xc = Xc + (32 * w + pi) * XS;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const float* src = g < 4 ? xp : xc;
    const floatx4 bx = *(const floatx4*)(src + 8 * (g & 3) + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 8 * g + 4 * h + j;
      acc_s = mfma32(Ws[k * WS + pi], bx[j], acc_s);
      acc_g = mfma32(Ws[k * WS + 32 + pi], bx[j], acc_g);
    }
  }
}

// ---- forward ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void layer_fwd_kernel(lbwn_layer_args a) {
  __shared__ __attribute__((aligned(16))) float sm[2 * LP * XS + 64 * WS + 32 * XS + 96];
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* Ws = Xc + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* br = bs + 64;
  const int tiles = (a.T + LP - 1) / LP;
  const int b = blockIdx.x / tiles, t0 = (blockIdx.x % tiles) * LP;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* xb = a.x_in + (long)b * (a.H + a.T) * a.Cr;
  stage_rows(Xp, xb, t0, -a.d, a.T, a.H, a.Cr, tid);
  stage_rows(Xc, xb, t0, 0, a.T, a.H, a.Cr, tid);
  stage_weights(Ws, Rs, bs, br, a, tid);
  __syncthreads();

  const int pi = lane & 31, h = lane >> 5;
  const int t = t0 + 32 * w + pi;
  const bool valid = t < a.T;
  floatx16 acc_s, acc_g;
  conv_tile(Xp, Xc, Ws, bs, a, b, t, valid, w, lane, acc_s, acc_g);
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = tanhf(acc_s[r]) * sigmoidf_(acc_g[r]);

  const long m = (long)b * a.T + t;
  if (a.x_out) {
    floatx16 acc_r;
    const float* xc = Xc + (32 * w + pi) * XS;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc_r[r] = xc[acc_row(r, h)] + br[acc_row(r, h)];
#pragma unroll
    for (int s = 0; s < 16; ++s) acc_r = mfma32(Rs[acc_row(s, h) * XS + pi], z[s], acc_r);
    if (valid) {
      float* xo = a.x_out + ((long)b * (a.H + a.T) + a.H + t) * a.Cr;
      if (a.Cr == 32) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          floatx4 v = {acc_r[4 * q], acc_r[4 * q + 1], acc_r[4 * q + 2], acc_r[4 * q + 3]};
          *(floatx4*)(xo + 8 * q + 4 * h) = v;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (acc_row(r, h) < a.Cr) xo[acc_row(r, h)] = acc_r[r];
      }
    }
  }
  if (valid) {
    float* zo = a.z + m * a.ldz;
    if (a.Cd == 32) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 v = {z[4 * q], z[4 * q + 1], z[4 * q + 2], z[4 * q + 3]};
        *(floatx4*)(zo + 8 * q + 4 * h) = v;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (acc_row(r, h) < a.Cd) zo[acc_row(r, h)] = z[r];
    }
  }
}

// ---- deferred slab reduction -------------------------------------------------------------

// Block `blk` of `nblk` reduces its share of the previous layer's per-block partials
// (fixed order -> deterministic) and writes the reference-layout gradients.
LBWN_DEV void reduce_slab_share(const lbwn_layer_args& a, int blk, int nblk, float* scratch, int tid) {
  const int ngroups = (SLAB + 31) / 32;
  for (int grp = blk; grp < ngroups; grp += nblk) {
    const int c = grp * 32 + (tid & 31);
    const int p0 = tid >> 5;
    float s = 0.f;
    if (c < SLAB)
      for (int p = p0; p < a.red_nparts; p += 8) s += a.red_slab[(long)p * a.red_stride + c];
    scratch[tid] = s;
    __syncthreads();
    if (tid < 32 && c < SLAB) {
      float tot = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) tot += scratch[j * 32 + tid];
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
    __syncthreads();
  }
}

// ---- backward ----------------------------------------------------------------------------

__global__ __launch_bounds__(256) void layer_bwd_kernel(lbwn_layer_args a) {
  __shared__ __attribute__((aligned(16)))
  float sm[3 * LP * XS + 64 * WS + 32 * XS + 96 + 4 * (32 * DS + 32 * XS) + 4 * 1024];
  float* Xp = sm;
  float* Xc = Xp + LP * XS;
  float* G = Xc + LP * XS;
  float* Ws = G + LP * XS;
  float* Rs = Ws + 64 * WS;
  float* bs = Rs + 32 * XS;
  float* br = bs + 64;
  float* DVall = br + 32;                 // 4 × [32][DS]
  float* ZTall = DVall + 4 * 32 * DS;     // 4 × [32][XS]
  const int tiles = (a.T + LP - 1) / LP;
  const int b = blockIdx.x / tiles, t0 = (blockIdx.x % tiles) * LP;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pi = lane & 31, h = lane >> 5;

  if (a.red_slab) reduce_slab_share(a, blockIdx.x, gridDim.x, DVall, tid);

  const float* xb = a.x_in + (long)b * (a.H + a.T) * a.Cr;
  stage_rows(Xp, xb, t0, -a.d, a.T, a.H, a.Cr, tid);
  stage_rows(Xc, xb, t0, 0, a.T, a.H, a.Cr, tid);
  if (a.g_a) {
    stage_plain(G, a.g_a, a.Cr, b, t0, 0, a.T, a.Cr, tid, false);
    __syncthreads();
    stage_plain(G, a.g_c0, a.Cr, b, t0, a.g_d, a.T, a.Cr, tid, true);
  } else {
    for (int e = tid; e < LP * XS; e += 256) G[e] = 0.f;
  }
  stage_weights(Ws, Rs, bs, br, a, tid);
  __syncthreads();

  const int t = t0 + 32 * w + pi;
  const bool valid = t < a.T;
  const long m = (long)b * a.T + t;

  // 1. recompute the gate
  floatx16 acc_s, acc_g;
  conv_tile(Xp, Xc, Ws, bs, a, b, t, valid, w, lane, acc_s, acc_g);
  floatx16 th, sg;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    th[r] = tanhf(acc_s[r]);
    sg[r] = sigmoidf_(acc_g[r]);
  }
  // 2. dzᵀ = dZskipᵀ + RES·gᵀ   (dz[pos][c] = dZ[pos][c] + Σ_o g[pos][o]·RES[c][o])
  floatx16 dz;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = acc_row(r, h);
    dz[r] = (valid && c < a.Cd) ? a.dz_skip[m * a.lddz + c] : 0.f;
  }
  const float* gp = G + (32 * w + pi) * XS;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const floatx4 gx = *(const floatx4*)(gp + 8 * g + 4 * h);
    const floatx4 rx = *(const floatx4*)(Rs + pi * XS + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) dz = mfma32(rx[j], gx[j], dz);
  }
  // 3. dvᵀ
  floatx16 dvs, dvg, z;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    z[r] = th[r] * sg[r];
    dvs[r] = dz[r] * sg[r] * (1.f - th[r] * th[r]);
    dvg[r] = dz[r] * th[r] * sg[r] * (1.f - sg[r]);
  }
  // park dv and z (pos-major) for the weight-grad products
  float* DV = DVall + w * 32 * DS;
  float* ZT = ZTall + w * 32 * XS;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    floatx4 v1 = {dvs[4 * q], dvs[4 * q + 1], dvs[4 * q + 2], dvs[4 * q + 3]};
    floatx4 v2 = {dvg[4 * q], dvg[4 * q + 1], dvg[4 * q + 2], dvg[4 * q + 3]};
    floatx4 v3 = {z[4 * q], z[4 * q + 1], z[4 * q + 2], z[4 * q + 3]};
    *(floatx4*)(DV + pi * DS + 8 * q + 4 * h) = v1;
    *(floatx4*)(DV + pi * DS + 32 + 8 * q + 4 * h) = v2;
    *(floatx4*)(ZT + pi * XS + 8 * q + 4 * h) = v3;
  }
  // 4. dx contributions: dcurᵀ = W1·dvᵀ (+ g), dprevᵀ = W0·dvᵀ   (rows = in channel)
  floatx16 acc_a, acc_c;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc_a[r] = gp[acc_row(r, h)];
    acc_c[r] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ko = 8 * q + 4 * h;
    const floatx4 w0s = *(const floatx4*)(Ws + pi * WS + ko);
    const floatx4 w0g = *(const floatx4*)(Ws + pi * WS + 32 + ko);
    const floatx4 w1s = *(const floatx4*)(Ws + (32 + pi) * WS + ko);
    const floatx4 w1g = *(const floatx4*)(Ws + (32 + pi) * WS + 32 + ko);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * q + j;
      acc_a = mfma32(w1s[j], dvs[s], acc_a);
      acc_a = mfma32(w1g[j], dvg[s], acc_a);
      acc_c = mfma32(w0s[j], dvs[s], acc_c);
      acc_c = mfma32(w0g[j], dvg[s], acc_c);
    }
  }
  if (valid) {
    float* oa = a.out_a + m * a.Cr;
    float* oc = a.out_c0 + m * a.Cr;
    if (a.Cr == 32) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 v1 = {acc_a[4 * q], acc_a[4 * q + 1], acc_a[4 * q + 2], acc_a[4 * q + 3]};
        floatx4 v2 = {acc_c[4 * q], acc_c[4 * q + 1], acc_c[4 * q + 2], acc_c[4 * q + 3]};
        *(floatx4*)(oa + 8 * q + 4 * h) = v1;
        *(floatx4*)(oc + 8 * q + 4 * h) = v2;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (acc_row(r, h) < a.Cr) {
          oa[acc_row(r, h)] = acc_a[r];
          oc[acc_row(r, h)] = acc_c[r];
        }
    }
  }
  __syncthreads();  // DV/ZT tiles of every wave visible

  // 5. optional dv export (LC grads) and GC table grads
  if (a.dv_out) {
    for (int e = lane; e < 32 * 64; e += 64) {
      const int p = e >> 6, o = e & 63, tt = t0 + 32 * w + p;
      const int oc = o & 31;
      if (tt < a.T && oc < a.Cd)
        a.dv_out[((long)b * a.T + tt) * a.lddv + (o < 32 ? oc : a.Cd + oc)] = DV[p * DS + o];
    }
  }
  if (a.gc_dtab) {
    const int tw0 = t0 + 32 * w;
    const int nv = min(32, a.T - tw0);
    if (nv > 0) {
      const int* idw = a.ids + (long)b * a.T + tw0;
      const int id0 = idw[0];
      bool uni = true;
      for (int p = 1; p < nv; ++p) uni &= (idw[p] == id0);
      const int o = lane, oc = o & 31;
      if (oc < a.Cd) {
        const int col = o < 32 ? oc : a.Cd + oc;
        if (uni) {
          float s = 0.f;
          for (int p = 0; p < nv; ++p) s += DV[p * DS + o];
          atomicAdd(a.gc_dtab + (long)id0 * 2 * a.Cd + col, s);
        } else {
          for (int p = 0; p < nv; ++p) atomicAdd(a.gc_dtab + (long)idw[p] * 2 * a.Cd + col, DV[p * DS + o]);
        }
      }
    }
  }

  // 6. weight-grad partials of this block: 5 tiles of 32×32 over K = 32 positions per wave,
  //    summed over the 4 waves in a fixed order through LDS (deterministic).
  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  float* RED = ZTall + 4 * 32 * XS;  // 4 × 1024 scratch
#pragma unroll 1
  for (int tile = 0; tile < 5; ++tile) {
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // tile 0: dSIG[0] (prev), 1: dSIG[1] (cur), 2: dGATE[0], 3: dGATE[1], 4: dRES.
    // A[i][k=pos] and B[k=pos][j] with k = 2s + h.
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int p = 2 * s + h;
      float av, bv;
      if (tile < 4) {
        const float* X = (tile & 1) ? Xc : Xp;
        av = X[(32 * w + p) * XS + pi];
        bv = DV[p * DS + (tile >> 1) * 32 + pi];
      } else {
        av = ZT[p * XS + pi];
        bv = G[(32 * w + p) * XS + pi];
      }
      acc = mfma32(av, bv, acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) RED[w * 1024 + acc_row(r, h) * 32 + pi] = acc[r];
    __syncthreads();
#pragma unroll
    for (int e = tid; e < 1024; e += 256)
      slab[tile * 1024 + e] = ((RED[e] + RED[1024 + e]) + RED[2048 + e]) + RED[3072 + e];
    __syncthreads();
  }
  // bias partials: dv column sums over the block's 128 positions, g column sums
  if (tid < 96) {
    float s = 0.f;
    if (tid < 64) {
      for (int ww = 0; ww < 4; ++ww)
        for (int p = 0; p < 32; ++p) s += DVall[ww * 32 * DS + p * DS + tid];
    } else {
      for (int p = 0; p < LP; ++p) s += G[p * XS + (tid - 64)];
    }
    slab[5120 + tid] = s;
  }
}

__global__ __launch_bounds__(256) void layer_reduce_kernel(lbwn_layer_args a) {
  __shared__ float scratch[256];
  reduce_slab_share(a, blockIdx.x, gridDim.x, scratch, threadIdx.x);
}

}  // namespace

int lbwn_layer_slab_stride() { return SLAB; }
int lbwn_layer_nblocks(int B, int T) { return B * ((T + LP - 1) / LP); }

static int check_layer(const lbwn_layer_args& a) {
  LBWN_REQUIRE(a.Cr >= 1 && a.Cr <= 32 && a.Cd >= 1 && a.Cd <= 32, "layer: n_res/n_dil must be in [1,32]");
  LBWN_REQUIRE(a.d >= 1 && a.d <= a.H, "layer: dilation %d exceeds halo %d", a.d, a.H);
  LBWN_REQUIRE(a.B >= 1 && a.T >= 1, "layer: empty batch");
  if (a.Cr == 32) LBWN_REQUIRE((((uintptr_t)a.x_in) & 15) == 0, "layer: x not 16-B aligned");
  return 0;
}

int lbwn_layer_fwd_launch(const lbwn_layer_args& a, hipStream_t st) {
  if (int e = check_layer(a)) return e;
  layer_fwd_kernel<<<lbwn_layer_nblocks(a.B, a.T), 256, 0, st>>>(a);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_bwd_launch(const lbwn_layer_args& a, hipStream_t st) {
  if (int e = check_layer(a)) return e;
  LBWN_REQUIRE(a.slab && a.slab_stride >= SLAB, "layer bwd: slab missing");
  layer_bwd_kernel<<<lbwn_layer_nblocks(a.B, a.T), 256, 0, st>>>(a);
  LBWN_CHECK_LAUNCH();
  return 0;
}

int lbwn_layer_reduce_launch(const lbwn_layer_args& a, hipStream_t st) {
  const int ngroups = (SLAB + 31) / 32;
  layer_reduce_kernel<<<ngroups, 256, 0, st>>>(a);
  LBWN_CHECK_LAUNCH();
  return 0;
}
