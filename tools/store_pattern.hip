// Diagnostic microbenchmark: HBM write bandwidth of observation-store patterns
// on several allocations of a 16-slot ring (as bench.py uses), to separate the
// cost of the store pattern from the kernels' own work.
//   tiles_k<TILE, NT>: each workgroup writes its TILE-row tile of K consecutive
//   ring slots (rollout_kernel's pattern); NT = nontemporal stores.
//   fill: one grid-stride launch per slot.
// Build (on the GPU box): hipcc --offload-arch=gfx950 -O3 -w -o store_pattern tools/store_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4 __attribute__((ext_vector_type(4)));

template <int TILE, bool NT>
__global__ __launch_bounds__(256) void tiles_k(uint8_t* ring, long slot, int R, int K, int row16, int rows) {
  const long base = (long)blockIdx.x * TILE * row16;
  const int total = (int)(min((long)TILE, (long)rows - (long)blockIdx.x * TILE) * row16);
  v4 z = {1u, 2u, 3u, 4u};
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot;
    for (int s = threadIdx.x; s < total; s += 256) {
      v4* p = reinterpret_cast<v4*>(out + (base + s) * 16);
      if (NT) __builtin_nontemporal_store(z, p);
      else *p = z;
    }
    __syncthreads();
  }
}

// each wave writes its own contiguous 1/FRONTS of the tile: FRONTS write fronts per workgroup
template <int TILE, int FRONTS>
__global__ __launch_bounds__(256) void tiles_fronts(uint8_t* ring, long slot, int R, int K, int row16) {
  const long base = (long)blockIdx.x * TILE * row16;
  const int total = TILE * row16;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int part = (total + FRONTS - 1) / FRONTS;
  const int f = wave % FRONTS, waves_per_front = 4 / FRONTS, wf = wave / FRONTS;
  const int lo = f * part, hi = min(total, lo + part);
  v4 z = {1u, 2u, 3u, 4u};
  for (int k = 0; k < K; ++k) {
    uint8_t* out = ring + (k % R) * slot;
    for (int s = lo + wf * 64 + lane; s < hi; s += 64 * waves_per_front)
      *reinterpret_cast<v4*>(out + (base + s) * 16) = z;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void fill(uint8_t* out, long n16) {
  v4 z = {1u, 2u, 3u, 4u};
  for (long s = blockIdx.x * 256L + threadIdx.x; s < n16; s += (long)gridDim.x * 256)
    *reinterpret_cast<v4*>(out + s * 16) = z;
}

int main() {
  const int rows = 65536, row16 = 101;     // 12x12 w=3: F = 404 fp32 = 101 x 16 B
  const long slot = (long)rows * row16 * 16;
  const int R = 16, K = 32, reps = 2;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<uint8_t*> rings;
  const char* names[] = {"tile64", "tile32", "tile128", "tile64_nt", "tile256", "fill", "t64_f2", "t64_f4", "t128_f4"};
  const bool contiguous = getenv("CONTIG") != nullptr;
  for (int i = 0; i < 6; ++i) {
    uint8_t* p;
    if (contiguous) {
      if (hipExtMallocWithFlags((void**)&p, slot * R, hipDeviceMallocContiguous) != hipSuccess) return 1;
    } else if (hipMalloc(&p, slot * R) != hipSuccess) {
      return 1;
    }
    rings.push_back(p);
    printf("ring %d:", i);
    for (int mode = 0; mode < 9; ++mode) {
      float ms = 0;
      for (int w = 0; w < 2; ++w) {
        (void)hipEventRecord(a);
        for (int r = 0; r < reps; ++r) {
          switch (mode) {
            case 0: tiles_k<64, false><<<rows / 64, 256>>>(p, slot, R, K, row16, rows); break;
            case 1: tiles_k<32, false><<<rows / 32, 256>>>(p, slot, R, K, row16, rows); break;
            case 2: tiles_k<128, false><<<rows / 128, 256>>>(p, slot, R, K, row16, rows); break;
            case 3: tiles_k<64, true><<<rows / 64, 256>>>(p, slot, R, K, row16, rows); break;
            case 4: tiles_k<256, false><<<rows / 256, 256>>>(p, slot, R, K, row16, rows); break;
            case 5: for (int k = 0; k < K; ++k) fill<<<2048, 256>>>(p + (k % R) * slot, slot / 16); break;
            case 6: tiles_fronts<64, 2><<<rows / 64, 256>>>(p, slot, R, K, row16); break;
            case 7: tiles_fronts<64, 4><<<rows / 64, 256>>>(p, slot, R, K, row16); break;
            default: tiles_fronts<128, 4><<<rows / 128, 256>>>(p, slot, R, K, row16); break;
          }
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      printf("  %s %.2f", names[mode], ms * 1e3 / (reps * K));
    }
    printf("  (us per slot)\n");
  }
  for (auto p : rings) (void)hipFree(p);
  return 0;
}
