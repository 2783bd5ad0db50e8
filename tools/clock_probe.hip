// In-kernel shader-clock probes (tuning tool, not product code; tools/clock_probe.py drives them).
//
// Two kernels shaped like the phased GEMM's halves (512 threads = 8 waves, one block per CU):
//   mfma_only  v_mfma_f32_16x16x32_f16 on operands held in registers (random data), 8 independent
//              accumulation chains per wave, no memory traffic in the loop
//   dma_only   the GEMM's per-K-step operand staging alone: 64 KiB per step (X + W panels of a 256 x 256
//              tile at BK = 64) by buffer_load ... lds (1 KiB per wave-instruction) into a 2-slot ring,
//              one barrier per step, no MFMAs
// Each block stamps s_memtime (shader clock) and s_memrealtime (100 MHz) at start and end into its own
// row of a stamp buffer; the clock it held is d(memtime) / d(realtime) x 100 MHz.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void stamp(unsigned long long* ts, int k) {
  if (threadIdx.x == 0) {
    ts[blockIdx.x * 4 + 2 * k] = __builtin_amdgcn_s_memtime();
    ts[blockIdx.x * 4 + 2 * k + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ __launch_bounds__(512) void mfma_only_kernel(const h8* __restrict__ src, float* __restrict__ sink,
                                                        unsigned long long* ts, int iters) {
  stamp(ts, 0);
  const int t = blockIdx.x * 512 + threadIdx.x;
  h8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = src[(t * 8 + i) & 65535];
    b[i] = src[(t * 8 + 4 + i) & 65535];
  }
  f4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; it += 2) {  // b index compile-time (a runtime one would go to scratch)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 3], b[i >> 2], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 3], b[2 + (i >> 2)], acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  sink[t] = s;
  __syncthreads();
  stamp(ts, 1);
}

__global__ __launch_bounds__(512) void dma_only_kernel(const _Float16* __restrict__ src, long src_bytes,
                                                       unsigned long long* ts, int steps) {
  __shared__ __attribute__((aligned(1024))) _Float16 ring[2][32768];  // 2 x 64 KiB
  stamp(ts, 0);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)src_bytes, 0x00020000);
  // each block walks its own 64-KiB-per-step window of the source (blocks of one XCD overlap the same
  // 8 MiB, as the GEMM's co-resident tiles share panels)
  const long span = src_bytes / 65536;
  const int b0 = (int)((blockIdx.x / 8) % (span > 128 ? 128 : span));
  auto issue = [&](int s) {
    const int slot = s & 1;
    const unsigned soff = (unsigned)((((long)b0 + s) % span) * 65536);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int piece = wave * 8 + j;  // 64 pieces of 1 KiB
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&ring[slot][piece * 512], 16,
                                               (int)(piece * 1024 + lane * 16), (int)soff, 0, 0);
    }
  };
  issue(0);
  for (int s = 0; s < steps; ++s) {
    if (s + 1 < steps) {
      issue(s + 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  stamp(ts, 1);
}

extern "C" int probe_mfma_only(const void* src, float* sink, unsigned long long* ts, int blocks, int iters,
                               void* stream) {
  hipLaunchKernelGGL(mfma_only_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream, (const h8*)src, sink, ts, iters);
  return (int)hipGetLastError();
}

extern "C" int probe_dma_only(const void* src, long src_bytes, unsigned long long* ts, int blocks, int steps,
                              void* stream) {
  hipLaunchKernelGGL(dma_only_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream, (const _Float16*)src, src_bytes,
                     ts, steps);
  return (int)hipGetLastError();
}
