// Which HW_ID fields tell two co-resident workgroups of a 2-blocks-per-CU kernel apart?
// hipcc --offload-arch=gfx950 -O3 tools/hwid_probe.hip -o /tmp/hwid && /tmp/hwid
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <map>
#include <vector>
__global__ __launch_bounds__(256, 2) void k(unsigned* o) {
  __shared__ float sm[13000];   // ~52 KB: two blocks per CU, as the split GEMM
  unsigned v, x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  sm[threadIdx.x] = v;
  __syncthreads();
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < 2000) {}
  if (threadIdx.x == 0) { o[2 * blockIdx.x] = v + (unsigned)sm[1] * 0; o[2 * blockIdx.x + 1] = x; }
}
int main() {
  unsigned* d; hipMalloc(&d, 2 * 512 * 4);
  k<<<512, 256>>>(d);
  std::vector<unsigned> h(1024);
  hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
  std::map<unsigned, std::vector<int>> cu;   // (xcc, se, sh, cu) -> blocks
  for (int b = 0; b < 512; ++b) {
    unsigned v = h[2 * b], x = h[2 * b + 1] & 0xf;
    unsigned key = (x << 16) | (((v >> 13) & 7) << 8) | (((v >> 12) & 1) << 4) | ((v >> 8) & 0xf);
    cu[key].push_back(b);
  }
  int shown = 0;
  for (auto& kv : cu) {
    if (shown++ < 12) {
      printf("xcc %u se %u sh %u cu %2u:", kv.first >> 16, (kv.first >> 8) & 7, (kv.first >> 4) & 1, kv.first & 0xf);
      for (int b : kv.second) printf("  blk %3d hwid %08x", b, h[2 * b]);
      printf("\n");
    }
  }
  printf("%zu distinct CUs\n", cu.size());
  return 0;
}
