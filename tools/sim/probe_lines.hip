// Host-only simulation: L2 requests of the giant-bitmap probes per 256-edge wave tile for two
// tile layouts — lane l holding edges 4l..4l+3 (probe instruction j = edges 4l+j, stride 4) and
// a transposed layout (instruction j = edges 64j..64j+63, consecutive) — over a canonical R-MAT
// list from the library's own generator function. A request = one distinct 64-B bitmap line
// (512 vertices) per wave instruction. Usage: probe_lines [scale]
#include "../../distributed_ghs_implementation_amd/csrc/ingest.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

namespace ghs {
void set_error(const std::string &) {}  // the library's error slot is not linked here
}

int main(int argc, char **argv) {
  const uint32_t scale = argc > 1 ? atoi(argv[1]) : 20;
  const uint64_t T = 16ull << scale;
  std::vector<uint64_t> k(T);
  for (uint64_t t = 0; t < T; ++t) k[t] = ghs::rmat_tuple(t, scale, 1);
  std::sort(k.begin(), k.end());
  k.erase(std::unique(k.begin(), k.end()), k.end());
  if (!k.empty() && k.back() == ((1ull << (2 * scale)) - 1ull)) k.pop_back();
  const uint64_t m = k.size(), mask = (1ull << scale) - 1;
  std::vector<uint32_t> v(m);
  for (uint64_t e = 0; e < m; ++e) v[e] = (uint32_t)(k[e] & mask);
  uint64_t req_stride = 0, req_trans = 0, instr = 0;
  std::vector<uint32_t> lines;
  for (uint64_t t0 = 0; t0 + 256 <= m; t0 += 256) {
    for (int j = 0; j < 4; ++j) {
      lines.clear();
      for (int l = 0; l < 64; ++l) lines.push_back(v[t0 + 4 * l + j] >> 9);
      std::sort(lines.begin(), lines.end());
      req_stride += std::unique(lines.begin(), lines.end()) - lines.begin();
      lines.clear();
      for (int l = 0; l < 64; ++l) lines.push_back(v[t0 + 64 * j + l] >> 9);
      std::sort(lines.begin(), lines.end());
      req_trans += std::unique(lines.begin(), lines.end()) - lines.begin();
      ++instr;
    }
  }
  printf("scale %u m %llu: requests per probe instruction  stride-4 %.2f  transposed %.2f  (of 64 lanes)\n", scale,
         (unsigned long long)m, (double)req_stride / instr, (double)req_trans / instr);
  return 0;
}
