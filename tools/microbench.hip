// Fundamental cost probes on gfx950 for the layer-kernel shape (256 blocks x 256 threads,
// one block per CU).  Build: hipcc -O3 --offload-arch=gfx950 tools/microbench.hip -o mb
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void k_empty(float* o) {
  if (threadIdx.x == 1000) o[0] = 1.f;
}

__global__ __launch_bounds__(256) void k_lds(float* o) {
  __shared__ float sm[36000];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 255] == -1.f) o[0] = 1.f;
}

template <int KB>
__global__ __launch_bounds__(256) void k_stage(const float* __restrict__ in, float* o) {
  __shared__ float sm[KB * 256];
  const floatx4* src = (const floatx4*)(in + (long)blockIdx.x * KB * 256);
  floatx4 v[KB / 4];
#pragma unroll
  for (int i = 0; i < KB / 4; ++i) v[i] = src[threadIdx.x + 256 * i];
#pragma unroll
  for (int i = 0; i < KB / 4; ++i) *(floatx4*)(sm + 4 * (threadIdx.x + 256 * i)) = v[i];
  __syncthreads();
  if (sm[(threadIdx.x * 7) & (KB * 256 - 1)] == -12345.f) o[0] = 1.f;
}

template <int N>
__global__ __launch_bounds__(256) void k_mfma(float* o) {
  floatx16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
#pragma unroll
  for (int i = 0; i < N; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  if (acc[3] == -1.f) o[0] = acc[0];
}

__global__ __launch_bounds__(256) void k_barriers(float* o) {
  __shared__ float sm[256];
  float v = threadIdx.x;
  for (int i = 0; i < 16; ++i) {
    sm[threadIdx.x] = v;
    __syncthreads();
    v += sm[(threadIdx.x + 1) & 255];
    __syncthreads();
  }
  if (v == -1.f) o[0] = v;
}

// straight-line code of N dependent-free VALU ops (≈8 B each): I-cache cold-fetch probe
template <int N>
__global__ __launch_bounds__(256) void k_code(float* o, float x) {
  float a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a0) : "v"(a1), "v"(a2));
  }
  if (a0 + a3 == -1.f) o[0] = a0;
}

// same independent-VALU work (4 accumulators) as straight-line code vs a small loop
template <int N>
__global__ __launch_bounds__(256) void k_line(float* o, float x) {
  float a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, b = x * 0.5f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile("v_fma_f32 %0, %4, %4, %0\n\tv_fma_f32 %1, %4, %4, %1\n\tv_fma_f32 %2, %4, %4, %2\n\tv_fma_f32 %3, %4, %4, %3"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b));
  }
  if (a0 + a1 + a2 + a3 == -1.f) o[0] = a0;
}
template <int N>
__global__ __launch_bounds__(256) void k_loop(float* o, float x, int iters) {
  float a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, b = x * 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      asm volatile("v_fma_f32 %0, %4, %4, %0\n\tv_fma_f32 %1, %4, %4, %1\n\tv_fma_f32 %2, %4, %4, %2\n\tv_fma_f32 %3, %4, %4, %3"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b));
    }
  }
  if (a0 + a1 + a2 + a3 == -1.f) o[0] = a0;
}

template <typename F>
float time_it(F f, int reps = 200) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) f();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  float *in, *o;
  (void)hipMalloc(&in, 256L * 64 * 1024 * 4);
  (void)hipMalloc(&o, 4096);
  (void)hipMemset(in, 0, 256L * 64 * 1024 * 4);
  printf("empty 256x256           %7.2f us/launch\n", time_it([&] { k_empty<<<256, 256>>>(o); }));
  printf("empty 1024x256          %7.2f us/launch\n", time_it([&] { k_empty<<<1024, 256>>>(o); }));
  printf("lds 144KB 256x256       %7.2f us/launch\n", time_it([&] { k_lds<<<256, 256>>>(o); }));
  printf("stage 16KB/blk 256x256  %7.2f us/launch\n", time_it([&] { k_stage<16><<<256, 256>>>(in, o); }));
  printf("stage 32KB/blk 256x256  %7.2f us/launch\n", time_it([&] { k_stage<32><<<256, 256>>>(in, o); }));
  printf("stage 64KB/blk 256x256  %7.2f us/launch\n", time_it([&] { k_stage<64><<<256, 256>>>(in, o); }));
  printf("mfma32x32x2 x64 256x256 %7.2f us/launch\n", time_it([&] { k_mfma<64><<<256, 256>>>(o); }));
  printf("mfma32x32x2 x224        %7.2f us/launch\n", time_it([&] { k_mfma<224><<<256, 256>>>(o); }));
  printf("32 barriers 256x256     %7.2f us/launch\n", time_it([&] { k_barriers<<<256, 256>>>(o); }));
  printf("4096 indep VALU straight (~32KB code) %7.2f us\n", time_it([&] { k_line<1024><<<256, 256>>>(o, 1.f); }));
  printf("4096 indep VALU loop 16x256 (~1KB)    %7.2f us\n", time_it([&] { k_loop<64><<<256, 256>>>(o, 1.f, 16); }));
  printf("2048 indep VALU straight (~16KB)      %7.2f us\n", time_it([&] { k_line<512><<<256, 256>>>(o, 1.f); }));
  printf("2048 indep VALU loop                  %7.2f us\n", time_it([&] { k_loop<64><<<256, 256>>>(o, 1.f, 8); }));
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("clock %d kHz, CUs %d\n", p.clockRate, p.multiProcessorCount);
  return 0;
}
