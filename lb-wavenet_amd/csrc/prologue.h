// Device bodies of the training step's independent start-of-step work, shared by their
// stand-alone kernels (misc.hip, gemm.hip) and by the fused step-prologue launch (layer.hip,
// lbwn_step_prologue_launch): each body walks its own index space over a range of `nblk` blocks
// of 256 threads, `blk` being this block's index within that range.
#pragma once
#include "common.h"

constexpr int PLANE_BK = 32;   // k per pre-split chunk (gemm.hip X3_BK)

// ---- D-separation state (tmodel.py:122-127, :165) -------------------------------------------
// SAVE for layer l (dilation d_l = 2^(l % nbl)) is [B][d_l][Cr], layers packed in order.
// x buffers: xall + l*xlayer_stride, per stream [H+T][Cr]; SAVE_l occupies rows [H-d, H).
// Rows of every layer's SAVE together (B·Σ_l d_l; Σ_{l'<l} d_{l'} = (l / nbl)·(2^nbl - 1) + 2^(l % nbl) - 1)
__host__ __device__ inline int dsep_rows(int L, int nbl, int B) {
  return ((L / nbl) * ((1 << nbl) - 1) + ((1 << (L % nbl)) - 1)) * B;
}

// Every layer's D-separation copy in ONE flat index space (32-bit; dsep_rows(...)·Cr < 2^31, checked
// by the launchers): packed row R = B·S(l) + b·d + i (S(l) = Σ_{l'<l} d_{l'}) holds SAVE elements
// [R·Cr, R·Cr + Cr), so the SAVE side is a straight run and only the x row needs the layer: within
// a run of nbl layers (B·(2^nbl - 1) rows) layer k starts at row B·(2^k - 1), so k = log2(w/B + 1).
// Float4 items when v4 (dsep_v4: Cr % 4 == 0, 16-B aligned buffers).  (Round 4 before: a block
// range per layer sized by the deepest d, 64-bit index division; the save took ~10 us for 5 MB at C2.)
template <bool TO_X>
LBWN_DEV void dsep_flat_body(long blk, long nblk, float* xall, long xls, float* save, int L, int nbl, int B, int T,
                             int H, int Cr, bool v4) {
  const int per = (1 << nbl) - 1, rows = dsep_rows(L, nbl, B);
  const int cw = v4 ? Cr >> 2 : Cr;   // items per row
  const int n = rows * cw;
  for (int e = (int)(blk * 256) + (int)threadIdx.x; e < n; e += (int)(nblk * 256)) {
    const int R = e / cw, c = e - R * cw;
    const int run = R / (B * per), w = R - run * (B * per);
    const int k = 31 - __builtin_clz(w / B + 1);
    const int local = w - B * ((1 << k) - 1);
    const int b = local >> k, i = local & ((1 << k) - 1), d = 1 << k;
    float* xr = xall + (long)(run * nbl + k) * xls + ((long)b * (H + T) + (TO_X ? H - d + i : H + T - d + i)) * Cr;
    float* sv = save + (long)R * Cr;
    if (v4) {
      if (TO_X) *(floatx4*)(xr + 4 * c) = *(const floatx4*)(sv + 4 * c);
      else *(floatx4*)(sv + 4 * c) = *(const floatx4*)(xr + 4 * c);
    } else {
      if (TO_X) xr[c] = sv[c];
      else sv[c] = xr[c];
    }
  }
}

inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }
inline bool dsep_v4(const float* xall, long xls, const float* save, int Cr) {
  return (Cr & 3) == 0 && (xls & 3) == 0 && al16(xall) && al16(save);
}
inline bool embed_v4(const float* pre, const float* pre_b, const float* x0, int Cr) {
  return (Cr & 3) == 0 && al16(pre) && (!pre_b || al16(pre_b)) && al16(x0);
}

// one-hot·PRE + PRE_BIAS == row gather (tmodel.py:53-66, :86-102), float4 items when v4
// (embed_v4), 32-bit indices (B·T·Cr < 2^31, checked by the launchers)
LBWN_DEV void embed_flat_body(long blk, long nblk, const int* __restrict__ q, const float* __restrict__ pre,
                              const float* pre_b, float* x0, int B, int T, int H, int Cr, int Q, bool v4) {
  const int cw = v4 ? Cr >> 2 : Cr;
  const int n = B * T * cw;
  for (int e = (int)(blk * 256) + (int)threadIdx.x; e < n; e += (int)(nblk * 256)) {
    const int m = e / cw, c = e - m * cw;
    const int b = m / T, t = m - b * T;
    int code = q[m];
    code = code < 0 ? 0 : (code >= Q ? Q - 1 : code);
    float* xo = x0 + ((long)b * (H + T) + H + t) * Cr;
    if (v4) {
      floatx4 v = *(const floatx4*)(pre + (long)code * Cr + 4 * c);
      if (pre_b) v += *(const floatx4*)(pre_b + 4 * c);
      *(floatx4*)(xo + 4 * c) = v;
    } else {
      float v = pre[(long)code * Cr + c];
      if (pre_b) v += pre_b[c];
      xo[c] = v;
    }
  }
}

LBWN_DEV void zero_body(long blk, long nblk, unsigned* p, long n) {
  for (long e = blk * 256 + threadIdx.x; e < n; e += nblk * 256) p[e] = 0u;
}

// Pre-split planes of weights W (f32, row stride ldw): out[r][kc][plane][32] = split of
// W[r][32·kc + j] (k-contiguous, trans = 0) or W[32·kc + j][r] (trans = 1); k ≥ K is zero.
// Up to 6 weights per launch.
struct SplitJobs {
  const float* W[6];
  long ldw[6];
  int rows[6], K[6], trans[6];
  unsigned short* out[6];
};
LBWN_DEV void split_planes_body(const SplitJobs& jb, int jj, long blk, long nblk) {
  const float* __restrict__ W = jb.W[jj];
  const long ldw = jb.ldw[jj];
  const int rows = jb.rows[jj], K = jb.K[jj], trans = jb.trans[jj];
  unsigned short* __restrict__ out = jb.out[jj];
  const int kch = (K + PLANE_BK - 1) / PLANE_BK;
  const long total = (long)rows * kch * (PLANE_BK / 2);   // pairs
  for (long e = blk * 256 + threadIdx.x; e < total; e += nblk * 256) {
    const int j2 = (int)(e % (PLANE_BK / 2)) * 2;
    const long rc = e / (PLANE_BK / 2);
    const int kc = (int)(rc % kch), r = (int)(rc / kch);
    const int k = kc * PLANE_BK + j2;
    floatx2 x;
    x[0] = k < K ? (trans ? W[(long)k * ldw + r] : W[(long)r * ldw + k]) : 0.f;
    x[1] = k + 1 < K ? (trans ? W[(long)(k + 1) * ldw + r] : W[(long)r * ldw + k + 1]) : 0.f;
    unsigned h, m, l;
    split2(x, h, m, l);
    unsigned* o = (unsigned*)(out + rc * (3 * PLANE_BK) + j2);
    o[0] = h;
    o[PLANE_BK / 2] = m;
    o[PLANE_BK] = l;
  }
}
