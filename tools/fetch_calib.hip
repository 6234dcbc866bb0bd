// FETCH_SIZE / WRITE_SIZE calibration for the access widths hs_rollout_kernel uses (MI355X_MICROARCH.md,
// HBM/rocprofv3: "other access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern"). One kernel per pattern over a buffer larger than the Infinity Cache, each launched
// once; tools/pmc_calib.py divides each dispatch's FETCH_SIZE / WRITE_SIZE by the bytes it moved.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/_build/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

// W-byte loads per lane, consecutive lanes consecutive (coalesced streaming)
template <class V>
__global__ void read_stream(const V* __restrict__ in, size_t n, double* __restrict__ sink) {
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const V v = in[i];
    const double* d = reinterpret_cast<const double*>(&v);
    for (int k = 0; k < (int)(sizeof(V) / sizeof(double)); k++) acc += d[k];
  }
  if (acc == 12345.678) sink[0] = acc;  // never true: keeps the loads
}

// the step kernel's record pattern: a lane reads R doubles of a 24-byte (3-double) entry at a
// per-lane record, records of one wavefront contiguous (the IK table rows: 6 limbs x 3 doubles)
__global__ void read_records3(const double* __restrict__ in, size_t n_rec, double* __restrict__ sink) {
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_rec; i += (size_t)gridDim.x * blockDim.x) {
    const double* e = in + 3 * i;
    acc += e[0] + e[1] + e[2];
  }
  if (acc == 12345.678) sink[0] = acc;
}

// output rows: a lane writes its rollout-step's 18 doubles (144 B, the tau row) at 144-byte stride
__global__ void write_rows18(double* __restrict__ out, size_t n_rows) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_rows; i += (size_t)gridDim.x * blockDim.x) {
    double* r = out + 18 * i;
    for (int k = 0; k < 18; k++) r[k] = (double)(i + k);
  }
}

// W-byte stores per lane, coalesced
template <class V>
__global__ void write_stream(V* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V v;
    double* d = reinterpret_cast<double*>(&v);
    for (int k = 0; k < (int)(sizeof(V) / sizeof(double)); k++) d[k] = (double)i;
    out[i] = v;
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB, four times the Infinity Cache
  void *buf, *out;
  double* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 0, bytes));
  CHECK(hipDeviceSynchronize());
  const dim3 grid(8192), block(256);
  hipLaunchKernelGGL(read_stream<double>, grid, block, 0, 0, (const double*)buf, bytes / 8, sink);
  hipLaunchKernelGGL(read_stream<double2>, grid, block, 0, 0, (const double2*)buf, bytes / 16, sink);
  hipLaunchKernelGGL(read_records3, grid, block, 0, 0, (const double*)buf, bytes / 24, sink);
  hipLaunchKernelGGL(write_stream<double>, grid, block, 0, 0, (double*)out, bytes / 8);
  hipLaunchKernelGGL(write_stream<double2>, grid, block, 0, 0, (double2*)out, bytes / 16);
  hipLaunchKernelGGL(write_rows18, grid, block, 0, 0, (double*)out, bytes / 144);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::printf("bytes per kernel: read_stream<double> %zu, read_stream<double2> %zu, read_records3 %zu, "
              "write_stream<double> %zu, write_stream<double2> %zu, write_rows18 %zu\n",
              bytes / 8 * 8, bytes / 16 * 16, bytes / 24 * 24, bytes / 8 * 8, bytes / 16 * 16, bytes / 144 * 144);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  CHECK(hipFree(sink));
  return 0;
}
