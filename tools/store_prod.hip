// Diagnostic microbenchmark: the rollout kernel's tick coupling without its
// work.  Workgroup = 1 "producer" wave that only spins for SPIN cycles per
// tick + 3 storing waves; one barrier per tick; tiles of ROWS rows of
// [65536][404] fp32, 16-slot ring, K = 32, 1024 workgroups over all tiles.
// SPIN = 0 shows the store path alone; SPIN > 0 shows what a producer of that
// latency costs when every tick waits for it.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_prod tools/store_prod.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int ROWS>
__global__ __launch_bounds__(256) void tiles(uint8_t* ring, long slot, int R, int K, int rowb, int ntiles, int spin) {
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x)
    for (int k = 0; k < K; ++k) {
      if (threadIdx.x < 64) {
        const long long t0 = clock64();
        while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
      } else {
        uint8_t* out = ring + (k % R) * slot + (long)t * ROWS * rowb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
        const int total = ROWS * rowb / 16;
        for (int s = threadIdx.x - 64; s < total; s += 192)
          __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
      }
      __syncthreads();
    }
}

int main() {
  const int rows = 65536, rowb = 1616;
  const long slot = (long)rows * rowb;
  const int R = 16, K = 32;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<uint8_t*> keep;
  const int spins[] = {0, 1000, 2000, 4000, 8000};
  for (int i = 0; i < 2; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    for (int rowsel = 0; rowsel < 3; ++rowsel) {
      const int ROWS = rowsel == 0 ? 16 : rowsel == 1 ? 32 : 64;
      printf("ring %d rows %d:", i, ROWS);
      for (int sp : spins) {
        float ms = 0;
        for (int w = 0; w < 2; ++w) {
          (void)hipEventRecord(a);
          if (ROWS == 16) tiles<16><<<1024, 256>>>(p, slot, R, K, rowb, 4096, sp);
          else if (ROWS == 32) tiles<32><<<1024, 256>>>(p, slot, R, K, rowb, 2048, sp);
          else tiles<64><<<1024, 256>>>(p, slot, R, K, rowb, 1024, sp);
          (void)hipEventRecord(b);
          (void)hipEventSynchronize(b);
          (void)hipEventElapsedTime(&ms, a, b);
        }
        printf("  spin %d: %.2f", sp, ms * 1e3 / K);
      }
      printf("  (us per slot)\n");
      fflush(stdout);
    }
  }
  for (auto p : keep) (void)hipFree(p);
  return 0;
}
