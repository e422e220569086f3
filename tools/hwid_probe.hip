// Where the rollout kernel's workgroups and waves land: 512 workgroups of 512 threads with the
// split kernel's LDS footprint (2 per CU), each wave recording HW_ID (SIMD, CU, SE, TG slot) and
// XCC_ID.  Prints how often the two workgroups of one CU start their wave 0 (the producer) on
// the same SIMD, and whether their TG slots differ in parity.
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/hwid_probe tools/hwid_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(512) void probe(unsigned* out) {
  extern __shared__ unsigned char smem[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);     // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
  if ((threadIdx.x & 63) == 0) {
    out[2 * (blockIdx.x * 8 + threadIdx.x / 64)] = hw;
    out[2 * (blockIdx.x * 8 + threadIdx.x / 64) + 1] = xcc;
  }
  smem[threadIdx.x] = (unsigned char)hw;
  const long long t0 = clock64();
  while (clock64() - t0 < 200000) __builtin_amdgcn_s_sleep(10);   // stay resident together
}

int main() {
  const int G = 512, W = 8;
  unsigned* d;
  if (hipMalloc(&d, G * W * 2 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(G), dim3(512), 42 * 1024, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(G * W * 2);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  // CU key: xcc, se, sh, cu
  std::map<unsigned, std::vector<int>> cu_wgs;
  int simd_hist[4][4] = {};
  for (int b = 0; b < G; ++b) {
    const unsigned hw = h[2 * b * W], xcc = h[2 * b * W + 1] & 0xf;
    const unsigned key = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
    cu_wgs[key].push_back(b);
    for (int w = 1; w < 4; ++w) simd_hist[w][(((h[2 * (b * W + w)] >> 4) & 3) - ((hw >> 4) & 3)) & 3]++;
  }
  int pairs = 0, same0 = 0, same01 = 0, tg_par_differs = 0, counts[8] = {};
  for (auto& kv : cu_wgs) {
    counts[kv.second.size() < 8 ? kv.second.size() : 7]++;
    if (kv.second.size() != 2) continue;
    const int a = kv.second[0], b = kv.second[1];
    const unsigned ha = h[2 * a * W], hb = h[2 * b * W];
    ++pairs;
    same0 += ((ha >> 4) & 3) == ((hb >> 4) & 3);
    same01 += ((h[2 * (a * W + 1)] >> 4) & 3) == ((hb >> 4) & 3);
    tg_par_differs += ((ha >> 16) & 1) != ((hb >> 16) & 1);
  }
  printf("CUs used %zu; WGs per CU histogram:", cu_wgs.size());
  for (int i = 0; i < 8; ++i) printf(" %d:%d", i, counts[i]);
  printf("\npairs %d: wave0 same SIMD %d, WG-A wave1 on WG-B wave0's SIMD %d, TG slot parity differs %d\n",
         pairs, same0, same01, tg_par_differs);
  for (int w = 1; w < 4; ++w)
    printf("wave %d SIMD offset from wave 0: %d %d %d %d\n", w, simd_hist[w][0], simd_hist[w][1],
           simd_hist[w][2], simd_hist[w][3]);
  for (int b = 0; b < 6; ++b) {
    printf("wg %d:", b);
    for (int w = 0; w < W; ++w) {
      const unsigned hw = h[2 * (b * W + w)];
      printf(" w%d simd%u cu%u se%u sh%u tg%u xcc%u |", w, (hw >> 4) & 3, (hw >> 8) & 0xf, (hw >> 13) & 7,
             (hw >> 12) & 1, (hw >> 16) & 0xf, h[2 * (b * W + w) + 1] & 0xf);
    }
    printf("\n");
  }
  return 0;
}
