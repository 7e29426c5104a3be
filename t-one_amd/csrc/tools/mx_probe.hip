// Probe of the v_mfma_scale_f32_16x16x128_f8f6f4 operand layout (e4m3, E8M0 scales): one wave, small
// integer operands placed by candidate lane->k maps, per-lane scales; prints the max error per map.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

__global__ void probe(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* D) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int w = 0; w < 8; ++w) {
    a[w] = *reinterpret_cast<const int*>(A + l * 32 + 4 * w);
    b[w] = *reinterpret_cast<const int*>(B + l * 32 + 4 * w);
  }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

static unsigned char enc(int v) {   // small integers -> e4m3 (exact for |v| <= 8)
  if (v == 0) return 0;
  const int s = v < 0 ? 0x80 : 0;
  int a = abs(v), e = 0;
  while ((a >> (e + 1)) > 0) ++e;            // a in [2^e, 2^(e+1))
  const int mant = ((a << 3) >> e) & 7;      // 3 mantissa bits
  return (unsigned char)(s | ((e + 7) << 3) | mant);
}

static int kmap(int m, int l, int j) {
  const int g = l >> 4;
  switch (m) {
    case 0: return 32 * g + j;
    case 1: return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
    case 2: return 8 * g + (j & 7) + 32 * (j >> 3);
    case 3: return 4 * g + (j & 3) + 16 * (j >> 2);
    default: return -1;
  }
}

int main() {
  int Am[16][128], Bm[128][16];
  srand(7);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) Am[i][k] = rand() % 7 - 3;
  for (int k = 0; k < 128; ++k) for (int j = 0; j < 16; ++j) Bm[k][j] = rand() % 7 - 3;
  unsigned char *dA, *dB; int *dsa, *dsb; float* dD;
  hipMalloc(&dA, 64 * 32); hipMalloc(&dB, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dD, 64 * 16);
  for (int sm = 0; sm < 4; ++sm)
  for (int m = 0; m < 4; ++m) {
    const int scl = 1;
    unsigned char hA[64 * 32], hB[64 * 32];
    int sa[64], sb[64];
    for (int l = 0; l < 64; ++l) {
      sa[l] = scl ? 125 + (l * l + 3 * l) % 5 : 127;   // 2^-2 .. 2^2
      sb[l] = scl ? 125 + (l * l * l + l / 7) % 5 : 127;
      for (int j = 0; j < 32; ++j) {
        hA[l * 32 + j] = enc(Am[l & 15][kmap(m, l, j)]);
        hB[l * 32 + j] = enc(Bm[kmap(m, l, j)][l & 15]);
      }
    }
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa, sizeof sa, hipMemcpyHostToDevice); hipMemcpy(dsb, sb, sizeof sb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dD);
    float hD[256];
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    double worst = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * (l >> 4) + r, col = l & 15;
        double ref = 0;
        for (int k = 0; k < 128; ++k) {
          // lane holding A[row][k]: l' = row + 16*g with kmap(m,l',j) == k
          double fa = 1, fb = 1;
          if (sm == 0) {          // the lane that holds the value
            for (int lp = row; lp < 64; lp += 16) for (int j = 0; j < 32; ++j) if (kmap(m, lp, j) == k) fa = ldexp(1.0, sa[lp] - 127);
            for (int lp = col; lp < 64; lp += 16) for (int j = 0; j < 32; ++j) if (kmap(m, lp, j) == k) fb = ldexp(1.0, sb[lp] - 127);
          } else if (sm == 1) {   // lane row + 16 * (k / 32)
            fa = ldexp(1.0, sa[row + 16 * (k >> 5)] - 127);
            fb = ldexp(1.0, sb[col + 16 * (k >> 5)] - 127);
          } else if (sm == 2) {   // lane 4 * row + k / 32
            fa = ldexp(1.0, sa[4 * row + (k >> 5)] - 127);
            fb = ldexp(1.0, sb[4 * col + (k >> 5)] - 127);
          } else {                // one scale per row: lane row
            fa = ldexp(1.0, sa[row] - 127);
            fb = ldexp(1.0, sb[col] - 127);
          }
          ref += Am[row][k] * fa * Bm[k][col] * fb;
        }
        worst = fmax(worst, fabs(hD[l * 4 + r] - ref));
      }
    printf("scale-map %d data-map %d: max |err| = %g\n", sm, m, worst);
  }
  return 0;
}
