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
LBWN_DEV long save_offset(int l, int nbl, int B, int Cr) {
  // Σ_{l'<l} d_{l'} = (l / nbl)·(2^nbl - 1) + (2^(l % nbl) - 1)
  const long s = (long)(l / nbl) * ((1L << nbl) - 1) + ((1L << (l % nbl)) - 1);
  return s * B * Cr;
}

template <bool TO_X>
LBWN_DEV void dsep_body(int l, long blk, long nblk, float* xall, long xls, float* save, int nbl, int B, int T, int H,
                        int Cr) {
  const int d = 1 << (l % nbl);
  const long n = (long)B * d * Cr;
  float* sv = save + save_offset(l, nbl, B, Cr);
  float* xl = xall + l * xls;
  for (long e = blk * 256 + threadIdx.x; e < n; e += nblk * 256) {
    const int c = (int)(e % Cr);
    const long r = e / Cr;
    const int i = (int)(r % d), b = (int)(r / d);
    if (TO_X) {
      xl[((long)b * (H + T) + (H - d + i)) * Cr + c] = sv[e];              // prepend
    } else {
      sv[e] = xl[((long)b * (H + T) + (H + T - d + i)) * Cr + c];          // save: last d rows of [SAVE ++ x]
    }
  }
}

// one-hot·PRE + PRE_BIAS == row gather (tmodel.py:53-66, :86-102)
LBWN_DEV void embed_body(long blk, long nblk, const int* __restrict__ q, const float* __restrict__ pre,
                         const float* pre_b, float* x0, int B, int T, int H, int Cr, int Q) {
  const long n = (long)B * T * Cr;
  for (long e = blk * 256 + threadIdx.x; e < n; e += nblk * 256) {
    const int c = (int)(e % Cr);
    const long m = e / Cr;
    const int b = (int)(m / T), t = (int)(m % T);
    int code = q[m];
    code = code < 0 ? 0 : (code >= Q ? Q - 1 : code);
    float v = pre[(long)code * Cr + c];
    if (pre_b) v += pre_b[c];
    x0[((long)b * (H + T) + H + t) * Cr + c] = v;
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
