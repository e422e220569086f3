// Diagnostic microbenchmark: where in its tile each workgroup starts writing.
// Rollout kernel pattern: 16-slot ring of [65536][404] fp32, K slots per launch,
// workgroup b writes its ROWS-row tile(s) of every slot (16-B stores, 256 threads).
//   rot<ROWS, UNIT>: start rotated by ((b * 37) mod pieces) * UNIT bytes, wrapping in the tile
//   multi<ROWS>: persistent, 2048 workgroups each owning tiles b, b + 2048, ...
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_rot tools/store_rot.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int ROWS, int UNIT>
__global__ __launch_bounds__(256) void rot(uint8_t* ring, long slot, int R, int K, int rowb) {
  const int total = ROWS * rowb / 16;
  const int pieces = ROWS * rowb / UNIT;
  const int r = UNIT ? (int)(((long)blockIdx.x * 37) % pieces) * (UNIT / 16) : 0;
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot + (long)blockIdx.x * ROWS * rowb;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
    for (int s = threadIdx.x; s < total; s += 256) {
      int q = s + r;
      if (q >= total) q -= total;
      __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, q * 16, 0, 0);
    }
    __syncthreads();
  }
}

template <int ROWS>
__global__ __launch_bounds__(256) void multi(uint8_t* ring, long slot, int R, int K, int rowb, int tiles) {
  const int total = ROWS * rowb / 16;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x)
    for (int k = 0; k < K; ++k) {
      uint8_t* out = ring + (k % R) * slot + (long)t * ROWS * rowb;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
      for (int s = threadIdx.x; s < total; s += 256)
        __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
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
  const char* names[] = {"t64", "t64rot256", "t64rot1k", "t64rot4k", "t16", "t16multi2048", "t16multi1024", "t32", "t32multi1024", "t32rot256"};
  std::vector<uint8_t*> keep;
  for (int i = 0; i < 4; ++i) {
    uint8_t* p;
    if (hipMalloc(&p, slot * R) != hipSuccess) return 1;
    keep.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 10; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        switch (mode) {
          case 0: rot<64, 0><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 1: rot<64, 256><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 2: rot<64, 1024><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 3: rot<64, 4096><<<rows / 64, 256>>>(p, slot, R, K, rowb); break;
          case 4: rot<16, 0><<<rows / 16, 256>>>(p, slot, R, K, rowb); break;
          case 5: multi<16><<<2048, 256>>>(p, slot, R, K, rowb, rows / 16); break;
          case 6: multi<16><<<1024, 256>>>(p, slot, R, K, rowb, rows / 16); break;
          case 7: rot<32, 0><<<rows / 32, 256>>>(p, slot, R, K, rowb); break;
          case 8: multi<32><<<1024, 256>>>(p, slot, R, K, rowb, rows / 32); break;
          default: rot<32, 256><<<rows / 32, 256>>>(p, slot, R, K, rowb); break;
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
