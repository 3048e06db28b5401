// randlat.hip -- random-access microbenchmark for the macro-atom walk's memory pattern on MI355X.
// Each lane follows a dependent chain of `hops` loads (the next address hashes the loaded value) through a
// table of `gib` GiB, optionally reading `width` consecutive doubles per hop.  Prints loads/s and latency.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__global__ void init(uint64_t *t, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    t[i] = (i * 0x9E3779B97F4A7C15ull) ^ (i >> 7);
}

template <int WIDTH>
__global__ void chase(const uint64_t *__restrict__ t, size_t n, int hops, uint64_t *out) {
  uint64_t x = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 0xD1B54A32D192ED03ull + 1;
  uint64_t acc = 0;
  for (int h = 0; h < hops; h++) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    const size_t i = (x % (n - WIDTH)) & ~(size_t)15;
    uint64_t v = 0;
#pragma unroll
    for (int w = 0; w < WIDTH; w++) v += t[i + w];
    x += v;
    acc += v;
  }
  if (acc == 42) out[0] = acc;
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 16;
  const int blocks = argc > 2 ? atoi(argv[2]) : 4096;
  const int hops = argc > 3 ? atoi(argv[3]) : 200;
  const size_t n = (size_t)(gib * (1ull << 30) / 8);
  uint64_t *t, *out;
  if (hipMalloc(&t, n * 8) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) { printf("alloc failed\n"); return 1; }
  init<<<4096, 256>>>(t, n);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int width : {1, 9}) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      if (width == 1) chase<1><<<blocks, 256>>>(t, n, hops, out);
      else chase<9><<<blocks, 256>>>(t, n, hops, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double lanes = (double)blocks * 256, hopsall = lanes * hops;
      if (rep) printf("table %.1f GiB lanes %.0f width %d: %.3f ms, %.2f G hops/s, %.2f us per hop per lane\n", gib, lanes,
                      width, ms, hopsall / ms / 1e6, ms * 1e3 / hops);
    }
  }
  return 0;
}
