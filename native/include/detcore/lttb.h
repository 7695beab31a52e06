// Largest-Triangle-Three-Buckets downsampling of metric series for charts (SURVEY M27;
// reference master/internal/lttb/lttb.go).  Keeps the first and last point; for each of the
// threshold-2 middle buckets picks the point forming the largest triangle with the previously
// selected point and the average of the next bucket.
#pragma once

#include <cstddef>
#include <vector>

namespace detcore {

struct Point {
  double x, y;
};

std::vector<Point> Downsample(const std::vector<Point>& data, size_t threshold);

}  // namespace detcore
