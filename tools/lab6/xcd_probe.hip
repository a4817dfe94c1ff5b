// Which XCD (HW_REG_XCC_ID) and CU does each workgroup of a 1024-thread, one-per-CU grid land on, and when does it
// start (s_memtime)?  Checks the round-robin-over-XCDs assumption behind bc_common.h xcd_remap.
//   hipcc --offload-arch=gfx950 -O2 tools/lab6/xcd_probe.hip -o /tmp/xcd_probe && /tmp/xcd_probe 4096 1024
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(unsigned* out, long long* t0, int spin) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
    t0[blockIdx.x] = __builtin_amdgcn_s_memtime();
  }
  long long s = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - s < spin) {
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int thr = argc > 2 ? atoi(argv[2]) : 1024;
  unsigned* d;
  long long* dt;
  if (hipMalloc(&d, 8 * n) != hipSuccess || hipMalloc(&dt, 8 * n) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(n), dim3(thr), 0, 0, d, dt, 20000);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(2 * n);
  std::vector<long long> ht(n);
  if (hipMemcpy(h.data(), d, 8 * n, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  if (hipMemcpy(ht.data(), dt, 8 * n, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  long long tmin = ht[0];
  for (int i = 0; i < n; ++i) tmin = ht[i] < tmin ? ht[i] : tmin;
  printf("wg xcc hw_id t0\n");
  for (int i = 0; i < n; ++i) printf("%d %u %08x %lld\n", i, h[2 * i] & 0xf, h[2 * i + 1], ht[i] - tmin);
  return 0;
}
