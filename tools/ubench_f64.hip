// Microbenchmark (tuning aid): cycles per fp64 FMA in a dependent chain and in 4 independent
// chains, for 1..4 wavefronts per SIMD; and the round trip of the rollout kernels' LDS exchange
// (ds_write, workgroup fence + s_barrier, ds_read) inside a one-wavefront workgroup.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_f64.hip -o tools/_build/ubench_f64 && tools/_build/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

__global__ __launch_bounds__(64) void chain1(double* out, double a, double b, long long* cyc) {
  double x = threadIdx.x * 1e-3;
  const long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; i++) x = fma(x, a, b);
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void chain4(double* out, double a, double b, long long* cyc) {
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  const long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; i++) {
    x0 = fma(x0, a, b);
    x1 = fma(x1, a, b);
    x2 = fma(x2, a, b);
    x3 = fma(x3, a, b);
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = x0 + x1 + x2 + x3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void lds_trip(double* out, long long* cyc) {
  __shared__ double s[64];
  double x = threadIdx.x;
  const long long t0 = clock64();
  for (int i = 0; i < 256; i++) {
    s[threadIdx.x] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    x = s[(threadIdx.x + 1) & 63] + 1.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int maxb = cus * 4 * 4;
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * 64 * maxb);
  hipMalloc(&cyc, sizeof(long long) * maxb);
  long long* h = new long long[maxb];
  auto avg = [&](int nb) {
    hipMemcpy(h, cyc, sizeof(long long) * nb, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nb; i++) s += h[i];
    return s / nb;
  };
  for (int w = 1; w <= 4; w++) {
    const int nb = cus * 4 * w;  // w wavefronts per SIMD (one-wavefront workgroups)
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    chain1<<<nb, 64>>>(out, 0.999, 1e-3, cyc);
    hipEventRecord(e0);
    chain1<<<nb, 64>>>(out, 0.999, 1e-3, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms1;
    hipEventElapsedTime(&ms1, e0, e1);
    const double c1 = avg(nb) / N;
    chain4<<<nb, 64>>>(out, 0.999, 1e-3, cyc);
    hipEventRecord(e0);
    chain4<<<nb, 64>>>(out, 0.999, 1e-3, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms4;
    hipEventElapsedTime(&ms4, e0, e1);
    const double c4 = avg(nb) / (4.0 * N);
    lds_trip<<<nb, 64>>>(out, cyc);
    hipDeviceSynchronize();
    lds_trip<<<nb, 64>>>(out, cyc);
    hipDeviceSynchronize();
    const double cl = avg(nb) / 512.0;
    printf("waves/SIMD %d: dependent fp64 FMA %.2f cyc/instr (%.1f us), 4 chains %.2f cyc/instr (%.1f us), "
           "LDS exchange round %.1f cyc\n", w, c1, ms1 * 1e3, c4, ms4 * 1e3, cl);
  }
  return 0;
}
