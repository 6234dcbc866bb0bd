#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const double* x, unsigned long long* bad, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  sincos(x[i], &s, &c);
  if (s != sin(x[i]) || c != cos(x[i])) atomicAdd(bad, 1ull);
}
int main() {
  const int n = 1 << 22;
  double* h = new double[n];
  uint64_t z = 12345;
  for (int i = 0; i < n; i++) {
    z += 0x9E3779B97F4A7C15ull; uint64_t v = z; v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull; v = (v ^ (v >> 27)) * 0x94D049BB133111EBull; v ^= v >> 31;
    double u = (v >> 11) * (1.0 / 9007199254740992.0);
    h[i] = (i % 4 == 0) ? (u - 0.5) * 20 : (i % 4 == 1) ? (u - 0.5) * 2000 : (i % 4 == 2) ? (u - 0.5) * 1e6 : (u - 0.5) * 7;
  }
  double* d; unsigned long long* b; hipMalloc(&d, n * 8); hipMalloc(&b, 8); hipMemset(b, 0, 8);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(d, b, n);
  unsigned long long bad = 0; hipMemcpy(&bad, b, 8, hipMemcpyDeviceToHost);
  printf("sincos mismatches: %llu of %d\n", bad, n);
  return bad != 0;
}
