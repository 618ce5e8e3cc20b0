// simd_placement.hip -- where the dispatcher puts the waves of a small workgroup: each wave
// records HW_ID (gfx9 layout: wave id [3:0], SIMD id [5:4], CU id [11:8], SE id [14:13]) and
// the XCC id, for workgroups of 2..8 waves, and of 2 and 4 waves with a register footprint
// that allows one wave per SIMD only (all 512 registers of the unified file claimed; a
// workgroup of 8 such waves cannot be resident, and its launch aborts the queue).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <bool BIG>
__global__ void where(unsigned *out) {
  if (BIG) asm volatile("" ::: "a255");  // 256 VGPRs + 256 AGPRs: one wave per SIMD
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
  // spin a little so that co-resident workgroups overlap
  long long t0 = clock64();
  while (clock64() - t0 < 200000) {
  }
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    out[2 * w] = hw;
    out[2 * w + 1] = xcc;
  }
}

int main() {
  unsigned *d;
  hipMalloc(&d, 2 * 64 * 8 * sizeof(unsigned));
  for (int big = 0; big < 2; ++big)
    for (int nw : {2, 4, 8}) {
      if (big && nw > 4) continue;  // 8 waves x 512 registers do not fit a CU
      const int grid = 8;
      hipMemset(d, 0xff, 2 * 64 * 8 * sizeof(unsigned));
      if (big)
        hipLaunchKernelGGL(where<true>, dim3(grid), dim3(64 * nw), 0, 0, d);
      else
        hipLaunchKernelGGL(where<false>, dim3(grid), dim3(64 * nw), 0, 0, d);
      hipDeviceSynchronize();
      std::vector<unsigned> h(2 * grid * nw);
      hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
      for (int b = 0; b < grid; ++b) {
        printf("big=%d waves=%d wg=%d:", big, nw, b);
        for (int w = 0; w < nw; ++w) {
          const unsigned hw = h[2 * (b * nw + w)];
          printf("  [xcc %u se %u cu %2u simd %u]", h[2 * (b * nw + w) + 1] & 0xf, (hw >> 13) & 3, (hw >> 8) & 15,
                 (hw >> 4) & 3);
        }
        printf("\n");
      }
    }
  hipFree(d);
  return 0;
}
