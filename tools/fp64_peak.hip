// fp64_peak -- measured FP64 FMA throughput of gfx950 (the compute roofline
// of the time-blocked sweep): ILP independent v_fma_f64 chains
// per lane, WPS waves per SIMD, every CU busy.
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_peak.hip -o tools/fp64_peak
#include <hip/hip_runtime.h>

#include <cstdio>

template <int ILP>
__global__ __launch_bounds__(64) void fma_kernel(double *out, int iters, double a, double b) {
  double x[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) x[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < ILP; ++i) x[i] = fma(x[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += x[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int ILP>
static void run(int waves_per_simd, int cus) {
  const int blocks = cus * 4 * waves_per_simd;
  double *out;
  (void)hipMalloc(&out, sizeof(double) * blocks * 64);
  const int iters = 4000;
  hipLaunchKernelGGL(fma_kernel<ILP>, dim3(blocks), dim3(64), 0, 0, out, 10, 0.999999, 1e-9);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(fma_kernel<ILP>, dim3(blocks), dim3(64), 0, 0, out, iters, 0.999999, 1e-9);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * ILP * (double)iters * blocks * 64;
  printf("ILP %2d  waves/SIMD %d  %8.3f ms  %7.2f TFLOP/s\n", ILP, waves_per_simd, ms, flops / ms / 1e9);
  (void)hipFree(out);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  for (int w : {1, 2, 4}) {
    run<1>(w, cus);
    run<2>(w, cus);
    run<4>(w, cus);
    run<8>(w, cus);
    run<16>(w, cus);
  }
  return 0;
}
