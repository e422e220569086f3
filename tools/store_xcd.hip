// Diagnostic microbenchmark: does the store rate of the rollout kernel's pattern
// depend on how many distinct pages each XCD writes at a time?  Same pattern as
// tools/store_rot.hip (16-slot ring of [65536][404] fp32, K slots per launch,
// 256 threads per workgroup, 16-B write-back stores), tiles assigned either
// round-robin over XCDs (block b -> tile b, so XCD b % 8 writes every 8th tile
// across the whole slot) or XCD-contiguous (block b -> tile (b % 8) * (B / 8) + b / 8,
// so each XCD writes one contiguous eighth of the slot).  The XCD of block b is
// b % 8 as the dispatcher is observed to place blocks (MI355X_MICROARCH.md);
// only speed depends on it.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_xcd tools/store_xcd.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int ROWS, bool XCD>
__global__ __launch_bounds__(256) void tiles(uint8_t* ring, long slot, int R, int K, int rowb, int ntiles) {
  const int B = gridDim.x;
  for (int tb = blockIdx.x; tb < ntiles; tb += B) {
    const int t = XCD ? ((tb % 8) * (ntiles / 8) + tb / 8) : tb;
    const int total = ROWS * rowb / 16;
    for (int k = 0; k < K; ++k) {
      uint8_t* out = ring + (k % R) * slot + (long)t * ROWS * rowb;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
      for (int s = threadIdx.x; s < total; s += 256)
        __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
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
  const char* names[] = {"t64", "t64xcd", "t16x1024", "t16x1024xcd", "t32x1024", "t32x1024xcd"};
  std::vector<uint8_t*> keep;
  for (int i = 0; i < 4; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 6; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: tiles<64, false><<<1024, 256>>>(p, slot, R, K, rowb, 1024); break;
          case 1: tiles<64, true><<<1024, 256>>>(p, slot, R, K, rowb, 1024); break;
          case 2: tiles<16, false><<<1024, 256>>>(p, slot, R, K, rowb, 4096); break;
          case 3: tiles<16, true><<<1024, 256>>>(p, slot, R, K, rowb, 4096); break;
          case 4: tiles<32, false><<<1024, 256>>>(p, slot, R, K, rowb, 2048); break;
          default: tiles<32, true><<<1024, 256>>>(p, slot, R, K, rowb, 2048); break;
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
