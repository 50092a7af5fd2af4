// Shared device/host helpers for the lbwn HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define LBWN_DEV __device__ __forceinline__

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
