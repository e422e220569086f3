// Diagnostic microbenchmark: store rate against the slot footprint written at a
// time.  B persistent workgroups of NT threads own 64-row tiles b, b + B, ...
// and write each tile for all K ticks before the next, so at any time the chip
// writes B tiles = B / 1024 of every slot.  Wave 0 optionally spins SPIN cycles
// per tick (a producer stand-in); the other waves store.  16-slot ring of
// [65536][404] fp32, 16-B write-back stores.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_fp tools/store_fp.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(NT) void tiles(uint8_t* ring, long slot, int R, int K, int rowb, int spin) {
  const int ntiles = 1024, ROWS = 64;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x)
    for (int k = 0; k < K; ++k) {
      if (threadIdx.x < 64 && spin > 0) {
        const long long t0 = clock64();
        while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
      } else {
        const int tid = spin > 0 ? threadIdx.x - 64 : threadIdx.x, nthr = spin > 0 ? NT - 64 : NT;
        uint8_t* out = ring + (k % R) * slot + (long)t * ROWS * rowb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
        const int total = ROWS * rowb / 16;
        for (int s = tid; s < total; s += nthr)
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
  for (int i = 0; i < 2; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    for (int spin : {0, 5000}) {
      printf("ring %d spin %d:", i, spin);
      for (int B : {256, 512, 1024}) {
        for (int nt : {512, 1024}) {
          float ms = 0;
          for (int w = 0; w < 2; ++w) {
            (void)hipEventRecord(a);
            if (nt == 512) tiles<512><<<B, 512>>>(p, slot, R, K, rowb, spin);
            else tiles<1024><<<B, 1024>>>(p, slot, R, K, rowb, spin);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms, a, b);
          }
          printf("  B%d x%d %.2f", B, nt, ms * 1e3 / K);
        }
      }
      printf("  (us per slot)\n");
      fflush(stdout);
    }
  }
  for (auto p : keep) (void)hipFree(p);
  return 0;
}
