// xcd_map.hip -- measurement tool (not product code): which XCD each
// workgroup of a 1-D grid runs on (HW_REG_XCC_ID), to check the blockIdx.x %
// 8 -> XCD assumption the unmask's and the encode's per-XCD run counters make.
//   hipcc --offload-arch=gfx950 -O2 -o tools/xcd_map tools/xcd_map.hip && tools/xcd_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_xcd(unsigned* out) {
  if (threadIdx.x == 0) {
    // HW_REG_XCC_ID (hwreg 20), bits [3:0]
    out[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
  }
}

int main() {
  const int grids[] = {256, 1024, 2048};
  for (int g : grids) {
    unsigned* d = nullptr;
    if (hipMalloc(&d, g * sizeof(unsigned)) != hipSuccess) return 1;
    k_xcd<<<g, 256>>>(d);
    std::vector<unsigned> h(g);
    if (hipMemcpy(h.data(), d, g * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int match = 0, counts[16] = {0};
    for (int b = 0; b < g; ++b) {
      match += (h[b] & 15u) == (unsigned)(b % 8);
      counts[h[b] & 15u]++;
    }
    printf("{\"grid\": %d, \"blockIdx_mod8_equals_xcc\": %d, \"per_xcc\": [", g, match);
    for (int x = 0; x < 8; ++x) printf("%d%s", counts[x], x < 7 ? ", " : "");
    printf("], \"first16\": [");
    for (int b = 0; b < 16; ++b) printf("%u%s", h[b], b < 15 ? ", " : "");
    printf("]}\n");
    (void)hipFree(d);
  }
  return 0;
}
