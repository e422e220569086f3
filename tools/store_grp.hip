// Diagnostic microbenchmark: 64 rows per workgroup per tick taken as G groups of
// 64/G rows spaced one region apart across workgroups (group j of workgroup b =
// rows 64/G * (b + B * j)), written group by group with a workgroup barrier
// between groups, so at each phase adjacent workgroups write adjacent regions
// (the spacing of 16-row tiles) while each keeps 64 envs.  16-slot ring of
// [65536][404] fp32, 1024 workgroups, 16-B write-back stores; SW storing waves.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_grp tools/store_grp.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int G, int SW>
__global__ __launch_bounds__(256) void grp(uint8_t* ring, long slot, int R, int K, int rowb) {
  const int B = gridDim.x, rows = 64 / G;
  const int tid = threadIdx.x - (4 - SW) * 64;
  const int per = rows * rowb / 16;
  for (int k = 0; k < K; ++k) {
    for (int j = 0; j < G; ++j) {
      if (tid >= 0) {
        uint8_t* out = ring + (k % R) * slot + (long)(blockIdx.x + (long)B * j) * rows * rowb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, rows * rowb, 0x00020000);
        for (int s = tid; s < per; s += SW * 64)
          __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
      }
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
  std::vector<uint8_t*> keep;
  const char* names[] = {"G1w4", "G4w4", "G4w3", "G2w3", "G1w3"};
  for (int i = 0; i < 4; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 5; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: grp<1, 4><<<1024, 256>>>(p, slot, R, K, rowb); break;
          case 1: grp<4, 4><<<1024, 256>>>(p, slot, R, K, rowb); break;
          case 2: grp<4, 3><<<1024, 256>>>(p, slot, R, K, rowb); break;
          case 3: grp<2, 3><<<1024, 256>>>(p, slot, R, K, rowb); break;
          default: grp<1, 3><<<1024, 256>>>(p, slot, R, K, rowb); break;
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
