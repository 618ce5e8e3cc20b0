// fp64_mix -- can gfx950's FP64 matrix core add throughput on top of the FP64 VALU?
// (the time-blocked sweep issues FP64 VALU at ~90% of the wave64 rate at
// the clock it holds; a block formulation of the per-line recurrence could move part of
// the work to v_mfma_f64_16x16x4_f64 only if the two pipes run concurrently at speed.)
// Measures, every CU busy:
//   valu  : ILP independent v_fma_f64 chains per lane
//   mfma  : 4 independent v_mfma_f64_16x16x4_f64 accumulators per wave
//   mixed : one wave issuing both streams, interleaved (MFMA executes while VALU issues)
//   split : even workgroups VALU, odd workgroups MFMA (two waves per SIMD)
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_mix.hip -o tools/fp64_mix
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

template <bool VALU, bool MFMA>
__device__ __forceinline__ void body(int iters, double a, double b, double *x, double4_t *c, double av, double bv) {
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (MFMA) {
#pragma unroll
        for (int m = 0; m < 4; ++m) c[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c[m], 0, 0, 0);
      }
      if (VALU) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = fma(x[i], a, b);
      }
    }
  }
}

// mode 0 valu, 1 mfma, 2 mixed (same wave), 3 split by workgroup parity
__global__ __launch_bounds__(64) void mix_kernel(double *out, int iters, int mode, double a, double b) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  double4_t c[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) c[m] = double4_t{0.0, 0.0, 0.0, 0.0};
  const double av = 1e-3 * threadIdx.x, bv = 0.5;
  int m = mode;
  if (mode == 3) m = (blockIdx.x & 1) ? 1 : 0;
  if (m == 0) body<true, false>(iters, a, b, x, c, av, bv);
  if (m == 1) body<false, true>(iters, a, b, x, c, av, bv);
  if (m == 2) body<true, true>(iters, a, b, x, c, av, bv);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
#pragma unroll
  for (int k = 0; k < 4; ++k) s += c[k][0] + c[k][1] + c[k][2] + c[k][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  // per iteration and wave: VALU 4 x 4 x 8 FMAs x 64 lanes; MFMA 4 x 4 x (16*16*4) FMAs
  const double valu_flops = 2.0 * 4 * 4 * 8 * 64, mfma_flops = 2.0 * 4 * 4 * 16 * 16 * 4;
  const char *names[] = {"valu", "mfma", "mixed", "split"};
  for (int wps : {1, 2}) {
    const int blocks = cus * 4 * wps;
    double *out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 64);
    for (int mode = 0; mode < 4; ++mode) {
      const int iters = 20000;
      hipLaunchKernelGGL(mix_kernel, dim3(blocks), dim3(64), 0, 0, out, 10, mode, 0.999999, 1e-9);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(mix_kernel, dim3(blocks), dim3(64), 0, 0, out, iters, mode, 0.999999, 1e-9);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      double per_wave = mode == 0 ? valu_flops : mode == 1 ? mfma_flops : mode == 2 ? valu_flops + mfma_flops
                                                                                    : 0.5 * (valu_flops + mfma_flops);
      const double flops = per_wave * iters * blocks;
      printf("%-6s waves/SIMD %d  %9.3f ms  %7.2f TFLOP/s\n", names[mode], wps, ms, flops / ms / 1e9);
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
    (void)hipFree(out);
  }
  return 0;
}
