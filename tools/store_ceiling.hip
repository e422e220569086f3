// Diagnostic microbenchmark: the write ceiling of the observation stream with
// the Infinity Cache (256 MiB) taken out of the picture.
//
// The rollout writes [65536][404] fp32 = 105.9 MB per tick into a ring of R
// slots.  A slot region is rewritten R ticks later; when the bytes written in
// between (the "reuse footprint") fit the Infinity Cache, dirty lines can be
// overwritten there before they reach HBM and a pattern looks faster than HBM
// allows.  Each pattern is timed with R = 16 and R = 64 (6.8 GB ring):
//   tiles<ROWS>  persistent workgroups, each owning tiles t = bid + j * grid and
//                writing one tile for all K ticks before the next (the rollout
//                kernel's unit order): reuse footprint = R * (grid tiles) rows;
//   tickmajor<ROWS> the same tiles, ticks outer: every tick covers the whole slot;
//   fill         one grid-stride launch per tick.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_ceiling tools/store_ceiling.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int ROWS, bool TICK_MAJOR>
__global__ __launch_bounds__(512) void tiles(uint8_t* ring, long slot, int R, int K, int rowb, int ntiles) {
  const int total = ROWS * rowb / 16;
  if (TICK_MAJOR) {
    for (int k = 0; k < K; ++k) {
      for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        uint8_t* out = ring + (long)(k % R) * slot + (long)t * ROWS * rowb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
        for (int s = threadIdx.x; s < total; s += 512)
          __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
      }
      __syncthreads();
    }
  } else {
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x)
      for (int k = 0; k < K; ++k) {
        uint8_t* out = ring + (long)(k % R) * slot + (long)t * ROWS * rowb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, ROWS * rowb, 0x00020000);
        for (int s = threadIdx.x; s < total; s += 512)
          __builtin_amdgcn_raw_buffer_store_b128(u4{1u, 2u, 3u, (unsigned)s}, rs, s * 16, 0, 0);
        __syncthreads();
      }
  }
}

__global__ __launch_bounds__(256) void fill(uint8_t* out, long n16) {
  const u4 z = {1u, 2u, 3u, 4u};
  for (long s = blockIdx.x * 256L + threadIdx.x; s < n16; s += (long)gridDim.x * 256)
    *reinterpret_cast<u4*>(out + s * 16) = z;
}

int main() {
  const int rows = 65536, rowb = 1616, K = 32;
  const long slot = (long)rows * rowb;
  uint8_t* p;
  if (hipMalloc(&p, slot * 64) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"tiles16", "tiles32", "tiles64", "tickmajor16", "tickmajor32", "tickmajor64", "fill"};
  for (int grid : {512, 1024}) {
    for (int R : {16, 64}) {
      printf("grid %4d R %2d:", grid, R);
      for (int mode = 0; mode < 7; ++mode) {
        std::vector<float> v;
        for (int rep = 0; rep < 5; ++rep) {
          float ms = 0;
          (void)hipEventRecord(a);
          switch (mode) {
            case 0: tiles<16, false><<<grid, 512>>>(p, slot, R, K, rowb, rows / 16); break;
            case 1: tiles<32, false><<<grid, 512>>>(p, slot, R, K, rowb, rows / 32); break;
            case 2: tiles<64, false><<<grid, 512>>>(p, slot, R, K, rowb, rows / 64); break;
            case 3: tiles<16, true><<<grid, 512>>>(p, slot, R, K, rowb, rows / 16); break;
            case 4: tiles<32, true><<<grid, 512>>>(p, slot, R, K, rowb, rows / 32); break;
            case 5: tiles<64, true><<<grid, 512>>>(p, slot, R, K, rowb, rows / 64); break;
            default:
              for (int k = 0; k < K; ++k) fill<<<2 * grid, 256>>>(p + (long)(k % R) * slot, slot / 16);
          }
          (void)hipEventRecord(b);
          (void)hipEventSynchronize(b);
          (void)hipEventElapsedTime(&ms, a, b);
          if (rep) v.push_back(ms * 1e3f / K);
        }
        std::sort(v.begin(), v.end());
        printf("  %s %.2f/%.2f", names[mode], v.front(), v[v.size() / 2]);
      }
      printf("  (us per slot: min/median; 105.9 MB per slot)\n");
      fflush(stdout);
    }
  }
  (void)hipFree(p);
  return 0;
}
