// linerate.hip -- random-line fetch rate of the MI355X memory system for the macro-atom walk's access shape.
// Every lane follows a dependent chain of hops; a hop reads W 16-byte chunks (W = 1, 2, 4, 8: 16 B .. one
// 128-byte line) at a random 128-byte-aligned offset of a table far larger than the Infinity Cache, and the
// next offset hashes the loaded data.  Reported per W and resident waves per SIMD: G hops/s (= lines/s) and
// the hop latency.  Usage: linerate [table GiB] [hops]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void init(u32x4 *t, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t h = (i * 0x9E3779B97F4A7C15ull) ^ (i >> 7);
    t[i] = u32x4{(unsigned)h, (unsigned)(h >> 32), (unsigned)(h * 3), (unsigned)(h >> 17)};
  }
}

template <int W>
__global__ __launch_bounds__(256) void chase(const u32x4 *__restrict__ t, size_t nlines, int hops, unsigned *out) {
  uint64_t x = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 0xD1B54A32D192ED03ull + 1;
  unsigned acc = 0;
  for (int h = 0; h < hops; h++) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    const u32x4 *p = t + (x % nlines) * 8;
    unsigned v = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const u32x4 c = p[w];
      v += c.x ^ c.y ^ c.z ^ c.w;
    }
    x += v;
    acc += v;
  }
  if (acc == 42u) out[0] = acc;
}

// the same 128-byte hops fetched cooperatively: wave instruction i has eight lanes read the eight 16-byte chunks
// of the line of lane 8i + (lane >> 3) (8 lines per instruction instead of 64), staged chunk-major in LDS
__global__ __launch_bounds__(256) void chase_coop(const u32x4 *__restrict__ t, size_t nlines, int hops, unsigned *out) {
  __shared__ u32x4 s[4][8][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t x = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 0xD1B54A32D192ED03ull + 1;
  unsigned acc = 0;
  for (int h = 0; h < hops; h++) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    const unsigned line = (unsigned)(x % nlines);
    u32x4 c[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const unsigned ls = (unsigned)__shfl((int)line, 8 * i + (lane >> 3), 64);
      c[i] = t[(size_t)ls * 8 + (lane & 7)];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) s[wv][lane & 7][8 * i + (lane >> 3)] = c[i];
    __builtin_amdgcn_wave_barrier();
    unsigned v = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
      const u32x4 d = s[wv][w][lane];
      v += d.x ^ d.y ^ d.z ^ d.w;
    }
    __builtin_amdgcn_wave_barrier();
    x += v;
    acc += v;
  }
  if (acc == 42u) out[0] = acc;
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 32;
  const int hops = argc > 2 ? atoi(argv[2]) : 400;
  const size_t nlines = (size_t)(gib * (1ull << 30) / 128);
  u32x4 *t;
  unsigned *out;
  if (hipMalloc(&t, nlines * 128) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  init<<<8192, 256>>>(t, nlines * 8);
  hipDeviceSynchronize();
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int waves : {2, 4, 8}) {
    const int blocks = ncu * waves;  // 256-thread blocks: `waves` resident waves per SIMD
    for (int w : {1, 2, 4, 8, 0}) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(a);
        if (w == 1) chase<1><<<blocks, 256>>>(t, nlines, hops, out);
        if (w == 2) chase<2><<<blocks, 256>>>(t, nlines, hops, out);
        if (w == 4) chase<4><<<blocks, 256>>>(t, nlines, hops, out);
        if (w == 8) chase<8><<<blocks, 256>>>(t, nlines, hops, out);
        if (w == 0) chase_coop<<<blocks, 256>>>(t, nlines, hops, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double lanes = (double)blocks * 256, all = lanes * hops;
        const int wb = w ? w : 8;
        if (rep)
          printf("table %.0f GiB waves/SIMD %d bytes/hop %3d%s: %8.3f ms  %6.2f G hops/s  %6.3f TB/s  %6.2f us/hop\n", gib,
                 waves, 16 * wb, w ? "" : " coop", ms, all / ms / 1e6, all * 16 * wb / ms / 1e9, ms * 1e3 / hops);
      }
    }
  }
  return 0;
}
