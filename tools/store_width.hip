// Diagnostic microbenchmark: bytes per lane per store instruction and cache
// policy for the rollout kernel's tile pattern (workgroup b writes rows
// [64b, 64b + 64) of each of K slots of a 16-slot ring of [65536][404] fp32),
// and 256-row tiles (fewer, longer write fronts).
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_width tools/store_width.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int BYTES, int POL, int ROWS, int NT>
__global__ __launch_bounds__(NT) void tilew(uint8_t* ring, long slot, int R, int K, int rowb) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const int total = ROWS * rowb / BYTES;          // stores per tile
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot + (long)blockIdx.x * ROWS * rowb;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
    for (int s = threadIdx.x; s < total; s += NT) {
      if (BYTES == 16) __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, POL);
      else if (BYTES == 8) __builtin_amdgcn_raw_buffer_store_b64(u2{1u, (unsigned)s}, rs, s * 8, 0, POL);
      else __builtin_amdgcn_raw_buffer_store_b32((unsigned)s, rs, s * 4, 0, POL);
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
  const char* names[] = {"w16", "w8", "w4", "w16nt", "w4nt", "w16x512", "r256w16", "r256w16x1024", "r16w16x256"};
  std::vector<uint8_t*> keep;
  for (int i = 0; i < 3; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 9; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: tilew<16, 0, 64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 1: tilew<8, 0, 64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 2: tilew<4, 0, 64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 3: tilew<16, 2, 64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 4: tilew<4, 2, 64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 5: tilew<16, 0, 64, 512><<<rows / 64, 512>>>(p, slot, R, K, rowb); break;
          case 6: tilew<16, 0, 256, 256><<<rows / 256, 256>>>(p, slot, R, K, rowb); break;
          case 7: tilew<16, 0, 256, 1024><<<rows / 256, 1024>>>(p, slot, R, K, rowb); break;
          default: tilew<16, 0, 16, 256><<<rows / 16, 256>>>(p, slot, R, K, rowb); break;
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
