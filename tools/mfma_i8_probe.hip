// Lane-map probe for v_mfma_i32_16x16x64_i8 on gfx950 (exact integer data, asymmetric A and B).
// Assumed: lane l holds A[l&15][16(l>>4) + j] and B[16(l>>4) + j][l&15] in byte j of its 16-byte
// operand; result register r of lane l is D[4(l>>4) + r][l&15]. Prints mismatches (0 = confirmed).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) {
    a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
    b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}
int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  for (int i = 0; i < 16; i++)
    for (int kk = 0; kk < 64; kk++) hA[i * 64 + kk] = (int8_t)(((i * 7 + kk * 3) % 23) - 11);
  for (int kk = 0; kk < 64; kk++)
    for (int j = 0; j < 16; j++) hB[kk * 16 + j] = (int8_t)(((kk * 5 + j * 11) % 19) - 9 + (j == 3 ? 60 : 0));
  int8_t *dA, *dB;
  int* dD;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dA, dB, dD);
  int hD[256];
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      int s = 0;
      for (int kk = 0; kk < 64; kk++) s += hA[i * 64 + kk] * hB[kk * 16 + j];
      if (s != hD[i * 16 + j]) bad++;
    }
  printf("mfma_i32_16x16x64_i8 lane-map mismatches: %d of 256\n", bad);
  return bad != 0;
}
