// repair.h -- OGR_G_Buffer(g, 0, 30) of a drill request geometry
// (worker/gdalprocess/drill.go:364-367), host side of drill_geom.cpp.
#pragma once
#include <vector>

namespace gsky {

// The zero-distance buffer of a Polygon / MultiPolygon given as rings
// (x / y, points per ring in `part`, the polygon of each ring in `poly`:
// its first ring is the shell, the others holes), as GEOS 3.7.2 computes it,
// written back into x / y / part as closed rings whose interior lies on their
// right.  Returns false, leaving the rings as drawn, when the buffer is empty
// (drill.go:365-367 then keeps the clone).
bool buffer0_rings(std::vector<double> &x, std::vector<double> &y, std::vector<int> &part,
                   const std::vector<int> &poly);

}  // namespace gsky
