// Diagnostic microbenchmark: observation-store patterns of a persistent tile
// kernel, K ticks over a 16-slot ring of [65536][404] fp32 (106 MB per slot).
//   tile<SW>:       workgroup b writes rows [64b, 64b + 64) of every slot
//   groups<G, SW>:  workgroup b writes G-row groups b, b + B, b + 2B, ... (B = workgroups):
//                   at any moment all workgroups write one dense region of the slot
//   SW = storing waves per 256-thread workgroup (4 = all; 3 = wave 0 idle, as the rollout kernel)
//   fill:           one grid-stride launch per slot
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_groups tools/store_groups.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int v4 __attribute__((ext_vector_type(4)));

template <int SW>
__global__ __launch_bounds__(256) void tile(uint8_t* ring, long slot, int R, int K, int row16) {
  const int t = threadIdx.x - (4 - SW) * 64;
  const long base = (long)blockIdx.x * 64 * row16;
  const int total = 64 * row16;
  v4 z = {1u, 2u, 3u, 4u};
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot;
    if (t >= 0)
      for (int s = t; s < total; s += SW * 64) *reinterpret_cast<v4*>(out + (base + s) * 16) = z;
    __syncthreads();
  }
}

template <int G, int SW>
__global__ __launch_bounds__(256) void groups(uint8_t* ring, long slot, int R, int K, int row16) {
  const int t = threadIdx.x - (4 - SW) * 64;
  const int per = G * row16;                     // 16-B stores per group
  v4 z = {1u, 2u, 3u, 4u};
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot;
    if (t >= 0)
      for (int j = 0; j < 64 / G; ++j) {
        const long base = ((long)j * gridDim.x + blockIdx.x) * per;
        for (int s = t; s < per; s += SW * 64) *reinterpret_cast<v4*>(out + (base + s) * 16) = z;
      }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void fill(uint8_t* out, long n16) {
  v4 z = {1u, 2u, 3u, 4u};
  for (long s = blockIdx.x * 256L + threadIdx.x; s < n16; s += (long)gridDim.x * 256)
    *reinterpret_cast<v4*>(out + s * 16) = z;
}

int main() {
  const int rows = 65536, row16 = 101;
  const long slot = (long)rows * row16 * 16;
  const int R = 16, K = 32, B = rows / 64;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"tile4", "tile3", "grp8w4", "grp8w3", "grp16w3", "grp32w3", "fill"};
  std::vector<uint8_t*> keep;
  for (int i = 0; i < 4; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 7; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: tile<4><<<B, 256>>>(p, slot, R, K, row16); break;
          case 1: tile<3><<<B, 256>>>(p, slot, R, K, row16); break;
          case 2: groups<8, 4><<<B, 256>>>(p, slot, R, K, row16); break;
          case 3: groups<8, 3><<<B, 256>>>(p, slot, R, K, row16); break;
          case 4: groups<16, 3><<<B, 256>>>(p, slot, R, K, row16); break;
          case 5: groups<32, 3><<<B, 256>>>(p, slot, R, K, row16); break;
          default: for (int k = 0; k < K; ++k) fill<<<2048, 256>>>(p + (k % R) * slot, slot / 16); break;
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      printf("  %s %.2f", names[mode], ms * 1e3 / K);
    }
    printf("  (us per slot)\n");
    fflush(stdout);
  }
  for (auto p : keep) (void)hipFree(p);
  return 0;
}
