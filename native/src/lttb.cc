#include "detcore/lttb.h"

#include <algorithm>
#include <cmath>

namespace detcore {

std::vector<Point> Downsample(const std::vector<Point>& data, size_t threshold) {
  if (threshold >= data.size() || threshold < 3) return data;
  std::vector<Point> out;
  out.reserve(threshold);
  const double every = static_cast<double>(data.size() - 2) / static_cast<double>(threshold - 2);
  size_t a = 0;
  out.push_back(data[0]);
  for (size_t i = 0; i < threshold - 2; ++i) {
    // average of the next bucket
    size_t avg_start = static_cast<size_t>(std::floor((i + 1) * every)) + 1;
    size_t avg_end = std::min(static_cast<size_t>(std::floor((i + 2) * every)) + 1, data.size());
    double ax = 0, ay = 0;
    for (size_t j = avg_start; j < avg_end; ++j) {
      ax += data[j].x;
      ay += data[j].y;
    }
    const double n = static_cast<double>(avg_end > avg_start ? avg_end - avg_start : 1);
    ax /= n;
    ay /= n;
    // pick the max-area point of this bucket
    size_t start = static_cast<size_t>(std::floor(i * every)) + 1;
    size_t end = static_cast<size_t>(std::floor((i + 1) * every)) + 1;
    double best = -1;
    size_t pick = start;
    for (size_t j = start; j < end && j < data.size(); ++j) {
      double area = std::fabs((data[a].x - ax) * (data[j].y - data[a].y) - (data[a].x - data[j].x) * (ay - data[a].y)) * 0.5;
      if (area > best) {
        best = area;
        pick = j;
      }
    }
    out.push_back(data[pick]);
    a = pick;
  }
  out.push_back(data.back());
  return out;
}

}  // namespace detcore
