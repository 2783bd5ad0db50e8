// VALU issue-rate probe (tuning tool, not product code): cycles per wave64 instruction for v_exp_f32,
// v_add_f32, v_fma_f32 and v_cvt_pk_f16_f32 chains, 1-8 waves per SIMD, by s_memtime around an unrolled
// loop of 8 independent chains x 16 instructions.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(1024) void rate_kernel(float* __restrict__ out, unsigned long long* __restrict__ cyc, int iters) {
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = -0.001f * (threadIdx.x + i);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(v[i]));
        if constexpr (OP == 1) asm volatile("v_add_f32 %0, %0, %0" : "+v"(v[i]));
        if constexpr (OP == 2) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v[i]));
        if constexpr (OP == 3) {
          float o;
          asm volatile("v_cvt_pk_f16_f32 %0, %1, %1" : "=v"(o) : "v"(v[i]));
          v[i] = o;
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int probe_rate(int op, int blocks, int threads, int iters, float* out, unsigned long long* cyc, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (op == 0) hipLaunchKernelGGL(rate_kernel<0>, dim3(blocks), dim3(threads), 0, st, out, cyc, iters);
  if (op == 1) hipLaunchKernelGGL(rate_kernel<1>, dim3(blocks), dim3(threads), 0, st, out, cyc, iters);
  if (op == 2) hipLaunchKernelGGL(rate_kernel<2>, dim3(blocks), dim3(threads), 0, st, out, cyc, iters);
  if (op == 3) hipLaunchKernelGGL(rate_kernel<3>, dim3(blocks), dim3(threads), 0, st, out, cyc, iters);
  return (int)hipGetLastError();
}
