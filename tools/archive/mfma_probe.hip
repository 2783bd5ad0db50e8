// Layout probe for the gfx950 f16 MFMA fragments and ds_read_b64_tr_b16 used by libvda.
// Exact small-integer data; prints PASS/FAIL per hypothesis.  Build:
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A: [16][32] row-major, B: [32][16] row-major, D: [16][16]
__global__ void p16(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}
// A: [32][16], B: [16][32], D: [32][32]
__global__ void p32(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 31) * 16 + 8 * (l >> 5) + j];
    b[j] = (_Float16)B[(8 * (l >> 5) + j) * 32 + (l & 31)];
  }
  f16v acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
}
// tr16: LDS image M[16][64] halfs with M[r][c] = r*64+c. Group g (16 lanes) reads rows 4g..4g+3,
// lane 4q+p supplies row 4g+q cols 4p..4p+3. Expect lane i of group to receive col i, element q = row 4g+q.
__global__ void ptr(float* out) {
  __shared__ _Float16 m[16 * 64];
  int l = threadIdx.x;
  for (int i = l; i < 16 * 64; i += 64) m[i] = (_Float16)i;
  __syncthreads();
  int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const _Float16* src = m + (4 * g + q) * 64 + 4 * p;
  s4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(src));
  h4 t = __builtin_bit_cast(h4, t0);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (float)t[e];
}

int main() {
  int fails = 0;
  {
    std::vector<float> A(16 * 32), B(32 * 16), D(256), R(256, 0);
    for (int i = 0; i < 16; ++i) for (int k = 0; k < 32; ++k) A[i * 32 + k] = (float)((i * 3 + k * 7) % 11 - 5);
    for (int k = 0; k < 32; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (float)((k * 5 + j * 13 + k * j) % 9 - 4);
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) for (int k = 0; k < 32; ++k) R[i * 16 + j] += A[i * 32 + k] * B[k * 16 + j];
    float *dA, *dB, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(p16, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 256; ++i) bad += (D[i] != R[i]);
    printf("mfma_f32_16x16x32_f16 layout: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad); fails += bad != 0;
    hipFree(dA); hipFree(dB); hipFree(dD);
  }
  {
    std::vector<float> A(32 * 16), B(16 * 32), D(1024), R(1024, 0);
    for (int i = 0; i < 32; ++i) for (int k = 0; k < 16; ++k) A[i * 16 + k] = (float)((i * 3 + k * 7) % 11 - 5);
    for (int k = 0; k < 16; ++k) for (int j = 0; j < 32; ++j) B[k * 32 + j] = (float)((k * 5 + j * 13 + k * j) % 9 - 4);
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) for (int k = 0; k < 16; ++k) R[i * 32 + j] += A[i * 16 + k] * B[k * 32 + j];
    float *dA, *dB, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(p32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 1024; ++i) bad += (D[i] != R[i]);
    printf("mfma_f32_32x32x16_f16 layout: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad); fails += bad != 0;
    hipFree(dA); hipFree(dB); hipFree(dD);
  }
  {
    float* dO; hipMalloc(&dO, 256 * 4);
    hipLaunchKernelGGL(ptr, dim3(1), dim3(64), 0, 0, dO);
    std::vector<float> O(256); hipMemcpy(O.data(), dO, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) { int g = l >> 4, i = l & 15;
      for (int e = 0; e < 4; ++e) if (O[l * 4 + e] != (float)((4 * g + e) * 64 + i)) ++bad; }
    printf("ds_read_b64_tr_b16 semantics: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad); fails += bad != 0;
    if (bad) { for (int l = 0; l < 20; ++l) printf("lane %d: %g %g %g %g\n", l, O[l*4], O[l*4+1], O[l*4+2], O[l*4+3]); }
    hipFree(dO);
  }
  printf("probe %s\n", fails ? "FAILED" : "OK");
  return fails ? 1 : 0;
}
