// Shared device/host helpers for the lbwn HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef unsigned uintx2 __attribute__((ext_vector_type(2)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

#define LBWN_DEV __device__ __forceinline__

// ---- f32 products on the bf16 matrix cores (gemm.hip header) ----------------
// x = hi + mid + lo exactly, each a bf16 (RN at every step; O(1) data, no subnormal terms).
LBWN_DEV unsigned pk_bf16(floatx2 v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
LBWN_DEV floatx2 unpk_bf16(unsigned p) { return (floatx2){__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)}; }
// Scalar subtractions on purpose: beside MFMAs a v_pk_add_f32 costs more issue time than two
// v_sub_f32 (MI355X_MICROARCH.md, filler prices), and the split runs between MFMAs.
LBWN_DEV void split2(floatx2 x, unsigned& h, unsigned& m, unsigned& l) {
  h = pk_bf16(x);
  float r0 = x[0] - __uint_as_float(h << 16), r1 = x[1] - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16((floatx2){r0, r1});
  r0 -= __uint_as_float(m << 16);
  r1 -= __uint_as_float(m & 0xffff0000u);
  l = pk_bf16((floatx2){r0, r1});
}
// 8 consecutive-k values (a = k 0..3, b = k 4..7) -> the three bf16x8 MFMA fragments
LBWN_DEV void split8(floatx4 a, floatx4 b, bf16x8 (&f)[3]) {
  unsigned h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
  split2((floatx2){a[0], a[1]}, h0, m0, l0);
  split2((floatx2){a[2], a[3]}, h1, m1, l1);
  split2((floatx2){b[0], b[1]}, h2, m2, l2);
  split2((floatx2){b[2], b[3]}, h3, m3, l3);
  f[0] = __builtin_bit_cast(bf16x8, (uintx4){h0, h1, h2, h3});
  f[1] = __builtin_bit_cast(bf16x8, (uintx4){m0, m1, m2, m3});
  f[2] = __builtin_bit_cast(bf16x8, (uintx4){l0, l1, l2, l3});
}
// acc += A·B over one 16-deep k-step from split fragments: the six products with i + j <= 2,
// small terms first
LBWN_DEV floatx16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// v_mfma_f32_32x32x2_f32: lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31];
// D[row=(r&3)+8*(r>>2)+4*(l>>5)][col=l&31] in accumulator register r (cdna_hip_programming §3).
LBWN_DEV floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row of accumulator register r for lane half h.
LBWN_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Gate transcendentals on the hardware v_exp_f32 / v_rcp_f32 (≈1 ulp each): σ(x) =
// 1/(1+e^-x); tanh(x) = 2σ(2x) - 1 (absolute error ≈1e-7, inside the 1e-5 parity bar).
LBWN_DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
LBWN_DEV float tanhf_(float x) { return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f; }
// The gate z = tanh(a)·σ(b) with ONE reciprocal (3 quarter-rate transcendentals instead of 4, on
// the chains' critical path): with E1 = e^-2a, E2 = e^-b, R = 1/((1+E1)(1+E2)):
// σ(b) = (1+E1)·R, z = (1-E1)·R.  a ≥ -20 and b ≥ -40 keep the product finite (tanh(-20) = -1 in
// f32; σ(-40) = 4e-18 stands for anything smaller, with z consistent with it).
LBWN_DEV float gate_zs(float a, float b, float& s) {
  const float e1 = __expf(-2.0f * fmaxf(a, -20.0f)), e2 = __expf(-fmaxf(b, -40.0f));
  const float p = 1.0f + e1, rr = __builtin_amdgcn_rcpf(p * (1.0f + e2));
  s = p * rr;
  return (1.0f - e1) * rr;
}
LBWN_DEV float gate_z(float a, float b) {
  float s;
  return gate_zs(a, b, s);
}

// Host-side error plumbing (defined in capi.cpp).
void lbwn_set_error(const char* fmt, ...);

#define LBWN_CHECK_LAUNCH()                                                     \
  do {                                                                          \
    hipError_t e__ = hipGetLastError();                                         \
    if (e__ != hipSuccess) {                                                    \
      lbwn_set_error("%s:%d: %s", __FILE__, __LINE__, hipGetErrorString(e__));  \
      return (int)e__;                                                          \
    }                                                                           \
  } while (0)

#define LBWN_REQUIRE(cond, ...)       \
  do {                                \
    if (!(cond)) {                    \
      lbwn_set_error(__VA_ARGS__);    \
      return 22; /* EINVAL */         \
    }                                 \
  } while (0)

#define LBWN_HIP(call)                                                          \
  do {                                                                          \
    hipError_t e__ = (call);                                                    \
    if (e__ != hipSuccess) {                                                    \
      lbwn_set_error("%s:%d: %s", __FILE__, __LINE__, hipGetErrorString(e__));  \
      return (int)e__;                                                          \
    }                                                                           \
  } while (0)
