// planet.cpp — the simulator's latency matrix (host side).
//
// Planet::from(dir) (fantoch/src/planet/mod.rs:38-54) reads one `<region>.dat`
// per region (Dat, planet/dat.rs:20-94): each line `min/avg/max/mdev:<to>`
// gives the average ping to <to>, truncated to whole milliseconds; the
// region's own line is replaced by 0 (INTRA_REGION_LATENCY, mod.rs:19).
// Planet::sorted orders every region's entries by (latency, region name)
// (mod.rs:122-140); the simulator only needs each region's position in that
// order (util.rs:159-167), so the loader exports it as a rank matrix.
// Regions are numbered in name order (Region derives Ord on its name,
// canonical C12).
#include <dirent.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "fantoch_amd.h"

namespace {

bool split_line(const std::string& line, double* avg, std::string* region) {
  // the reference splits on '/' and ':' and takes the 2nd and the last field
  size_t fields = 0, start = 0;
  std::string second, last;
  for (size_t i = 0; i <= line.size(); ++i) {
    if (i == line.size() || line[i] == '/' || line[i] == ':') {
      const std::string f = line.substr(start, i - start);
      if (fields == 1) second = f;
      last = f;
      ++fields;
      start = i + 1;
    }
  }
  if (fields < 3) return false;
  char* end = nullptr;
  *avg = std::strtod(second.c_str(), &end);
  if (end == second.c_str()) return false;
  *region = last;
  return true;
}

}  // namespace

extern "C" int fx_planet_load(const char* dir, uint32_t cap, uint32_t* num_regions, char* names,
                              uint32_t names_bytes, uint16_t* ping, uint8_t* rank) {
  if (!dir || !num_regions) return FX_ERR_INVALID_ARG;
  DIR* d = opendir(dir);
  if (!d) return FX_ERR_INVALID_ARG;
  std::vector<std::string> regions;
  while (dirent* e = readdir(d)) {
    const std::string f = e->d_name;
    if (f.size() > 4 && f.compare(f.size() - 4, 4, ".dat") == 0) regions.push_back(f.substr(0, f.size() - 4));
  }
  closedir(d);
  std::sort(regions.begin(), regions.end());
  const uint32_t R = (uint32_t)regions.size();
  *num_regions = R;
  if (R == 0 || R > 255) return FX_ERR_INVALID_ARG;
  if (!ping || !rank) return FX_OK;  // size query
  if (cap < R) return FX_ERR_CAPACITY;
  std::vector<int64_t> lat((size_t)R * R, -1);
  for (uint32_t a = 0; a < R; ++a) {
    std::ifstream in(std::string(dir) + "/" + regions[a] + ".dat");
    if (!in) return FX_ERR_INVALID_ARG;
    std::string line;
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      double avg = 0;
      std::string to;
      if (!split_line(line, &avg, &to)) return FX_ERR_INVALID_ARG;
      auto it = std::lower_bound(regions.begin(), regions.end(), to);
      if (it == regions.end() || *it != to) return FX_ERR_INVALID_ARG;
      const uint32_t b = (uint32_t)(it - regions.begin());
      lat[(size_t)a * R + b] = b == a ? 0 : (int64_t)avg;
    }
  }
  for (uint32_t a = 0; a < R; ++a) {
    std::vector<std::pair<int64_t, uint32_t>> v;
    for (uint32_t b = 0; b < R; ++b) {
      const int64_t l = lat[(size_t)a * R + b];
      if (l < 0 || l > 0xFFFF) return FX_ERR_INVALID_ARG;  // every pair must be known
      ping[(size_t)a * cap + b] = (uint16_t)l;
      v.push_back({l, b});
    }
    std::sort(v.begin(), v.end());  // (latency, name): b ascending is name order
    for (uint32_t i = 0; i < R; ++i) rank[(size_t)a * cap + v[i].second] = (uint8_t)i;
  }
  if (names && names_bytes) {
    std::string all;
    for (auto& r : regions) all += r + "\n";
    std::strncpy(names, all.c_str(), names_bytes - 1);
    names[names_bytes - 1] = 0;
  }
  return FX_OK;
}
