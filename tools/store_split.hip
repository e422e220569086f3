// Diagnostic microbenchmark: 64-row tiles per workgroup (1024 workgroups x 256
// threads, 16-slot ring of [65536][404] fp32, 16-B write-back stores), each
// tick's tile written in S phases of 64/S rows with a workgroup barrier between
// phases, against 16-row tiles.  Separates "bytes per workgroup per barrier"
// from "bytes per workgroup per tick".
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_split tools/store_split.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int ROWS, int S, int NT>
__global__ __launch_bounds__(NT) void tiles(uint8_t* ring, long slot, int R, int K, int rowb, int ntiles) {
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x)
    for (int k = 0; k < K; ++k) {
      uint8_t* out = ring + (k % R) * slot + (long)t * ROWS * rowb;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
      const int part = ROWS / S * rowb / 16;
      for (int p = 0; p < S; ++p) {
        for (int s = threadIdx.x; s < part; s += NT)
          __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, (p * part + s) * 16, 0, 0);
        __syncthreads();
      }
    }
}

int main() {
  const int rows = 65536, rowb = 1616;
  const long slot = (long)rows * rowb;
  const int R = 16, K = 32;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"t64s1", "t64s4", "t64s1x512", "t64s4x512", "t16", "t64s2"};
  std::vector<uint8_t*> keep;
  for (int i = 0; i < 3; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 6; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: tiles<64, 1, 256><<<1024, 256>>>(p, slot, R, K, rowb, 1024); break;
          case 1: tiles<64, 4, 256><<<1024, 256>>>(p, slot, R, K, rowb, 1024); break;
          case 2: tiles<64, 1, 512><<<1024, 512>>>(p, slot, R, K, rowb, 1024); break;
          case 3: tiles<64, 4, 512><<<1024, 512>>>(p, slot, R, K, rowb, 1024); break;
          case 4: tiles<16, 1, 256><<<1024, 256>>>(p, slot, R, K, rowb, 4096); break;
          default: tiles<64, 2, 256><<<1024, 256>>>(p, slot, R, K, rowb, 1024); break;
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
