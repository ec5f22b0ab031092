// apg_scan.hpp — exact LIDAR segment scan on device (one lane = one segment).
//
// Replaces LIDARLocalization2DEnv.__lidar_scan (ap_gym/envs/lidar_localization2d.py:496-536), i.e.
// shapely.LineString([p, q]).intersection(union_all(unit boxes)) followed by the reference's
// branch on the GEOS result type.  Semantics (DESIGN.md §LIDAR-scan semantics): the segment is
// noded at every boundary point of the closed union U it meets (edge crossings, boundary lattice
// vertices); noded pieces inside U are LineStrings, boundary nodes with no adjacent inside piece
// are Points; the result type decides the distance:
//   empty -> |q-p| (f32)         LineString -> max(|c-p|_f64 - 1e-3, 0)    Point -> 0
//   Multi* -> max(min_i |f32(c_i)-p|_f32 - 1e-3f, 0)                    mixed -> |q-p| (f32)
//
// Algorithm: a DDA walk over grid-line crossings in segment order.  Crossing order uses the exact
// orientation predicate (filter + exact fallback); occupancy comes from an accessor `occ.at(x, y)`
// (cells outside the map are free); GEOS's crossing coordinate is only computed for the node that
// starts a line piece.
#pragma once
#include "apg_device.hpp"

namespace apg {

enum : int { SCAN_EMPTY = 0, SCAN_LINE = 1, SCAN_MULTILINE = 2, SCAN_POINT = 3, SCAN_MULTIPOINT = 4,
             SCAN_COLLECTION = 5 };

struct ScanOut {
  float dist;
  int kind;
};

template <class Occ>
APG_DEV void closure_status(const Occ &occ, int i0, int i1, int j0, int j1, bool &in_u, bool &all) {
  bool any = false, al = true;
  for (int i = i0; i <= i1; i++)
    for (int j = j0; j <= j1; j++) {
      const bool o = occ.at(i, j);
      any |= o;
      al &= o;
    }
  in_u = any;
  all = al;
}

template <class Occ>
APG_DEV ScanOut lidar_scan(const Occ &occ, float fpx, float fpy, float fqx, float fqy) {
  const double px = fpx, py = fpy, qx = fqx, qy = fqy;
  const int sx = (fqx > fpx) - (fqx < fpx), sy = (fqy > fpy) - (fqy < fpy);
  const float flpx = floorf(fpx), flpy = floorf(fpy), flqx = floorf(fqx), flqy = floorf(fqy);
  const bool pxi = flpx == fpx, pyi = flpy == fpy, qxi = flqx == fqx, qyi = flqy == fqy;
  const int ipx = (int)flpx, ipy = (int)flpy, iqx = (int)flqx, iqy = (int)flqy;
  // integer lines strictly inside the segment
  int ax = 0, nxl = 0, by = 0, nyl = 0;
  if (sx > 0) {
    ax = ipx + 1;
    nxl = (qxi ? iqx - 1 : iqx) - ax + 1;
  } else if (sx < 0) {
    ax = pxi ? ipx - 1 : ipx;
    nxl = ax - (iqx + 1) + 1;
  }
  if (sy > 0) {
    by = ipy + 1;
    nyl = (qyi ? iqy - 1 : iqy) - by + 1;
  } else if (sy < 0) {
    by = pyi ? ipy - 1 : ipy;
    nyl = by - (iqy + 1) + 1;
  }
  if (nxl < 0) nxl = 0;
  if (nyl < 0) nyl = 0;
  const bool colv = sx == 0 && pxi, colh = sy == 0 && pyi;
  int cx = (sx < 0 && pxi) ? ipx - 1 : ipx;
  int cy = (sy < 0 && pyi) ? ipy - 1 : ipy;

  auto ivl_in = [&](int x, int y) -> bool {
    if (colv) return occ.at(x - 1, y) | occ.at(x, y);
    if (colh) return occ.at(x, y - 1) | occ.at(x, y);
    return occ.at(x, y);
  };

  // previous node: type 0 = p, 1 = lattice (a, b), 2 = x-crossing on edge (a, b)-(a, b+1),
  // 3 = y-crossing on edge (a, b)-(a+1, b)
  int pv_t = 0, pv_a = 0, pv_b = 0;
  bool pv_onb, pv_left_in = false;
  {
    bool in_u, all;
    closure_status(occ, pxi ? ipx - 1 : ipx, ipx, pyi ? ipy - 1 : ipy, ipy, in_u, all);
    pv_onb = in_u && !all;
  }
  bool cur_in = ivl_in(cx, cy);
  int n_lines = 0, n_points = 0;
  double l0x = 0.0, l0y = 0.0;
  float best_line = __builtin_inff(), best_point = __builtin_inff();

  auto node_coord = [&](int t, int a, int b, double &x, double &y) {
    if (t == 0) {
      x = px;
      y = py;
    } else if (t == 1) {
      x = (double)a;
      y = (double)b;
    } else if (t == 2) {
      geos_intersection(px, py, qx, qy, (double)a, (double)b, (double)a, (double)(b + 1), x, y);
    } else if (t == 3) {
      geos_intersection(px, py, qx, qy, (double)a, (double)b, (double)(a + 1), (double)b, x, y);
    } else {
      x = qx;
      y = qy;
    }
  };
  auto dist_f32 = [&](double x, double y) -> float {
    return norm_f32(__fsub_rn((float)x, fpx), __fsub_rn((float)y, fpy));
  };
  // close the piece [prev node, new node]
  auto close_piece = [&]() {
    if (cur_in) {
      double x, y;
      node_coord(pv_t, pv_a, pv_b, x, y);
      if (++n_lines == 1) {
        l0x = x;
        l0y = y;
      }
      best_line = fminf(best_line, dist_f32(x, y));
    } else if (pv_onb && !pv_left_in) {
      double x, y;
      node_coord(pv_t, pv_a, pv_b, x, y);
      n_points++;
      best_point = fminf(best_point, dist_f32(x, y));
    }
    pv_left_in = cur_in;
  };

  int xi = 0, yi = 0;
  while (xi < nxl || yi < nyl) {
    const int a = ax + sx * xi, b = by + sy * yi;
    bool takex, takey;
    if (xi < nxl && yi < nyl) {
      // sign(t_a - t_b) = -orient(p, q, (a, b)) * sx * sy
      const int c = -orient(px, py, qx, qy, (double)a, (double)b) * sx * sy;
      takex = c <= 0;
      takey = c >= 0;
    } else {
      takex = xi < nxl;
      takey = !takex;
    }
    int et, ea, eb, i0, i1, j0, j1;
    if ((takex && takey) || (takex && colh) || (takey && colv)) {
      et = 1;
      ea = takex ? a : ipx;
      eb = takey ? b : ipy;
      i0 = ea - 1;
      i1 = ea;
      j0 = eb - 1;
      j1 = eb;
    } else if (takex) {
      et = 2;
      ea = a;
      eb = cy;
      i0 = a - 1;
      i1 = a;
      j0 = j1 = cy;
    } else {
      et = 3;
      ea = cx;
      eb = b;
      i0 = i1 = cx;
      j0 = b - 1;
      j1 = b;
    }
    bool in_u, all;
    closure_status(occ, i0, i1, j0, j1, in_u, all);
    if (takex) {
      cx += sx;
      xi++;
    }
    if (takey) {
      cy += sy;
      yi++;
    }
    if (in_u && !all) {  // boundary point => node
      close_piece();
      pv_t = et;
      pv_a = ea;
      pv_b = eb;
      pv_onb = true;
    }
    cur_in = ivl_in(cx, cy);
  }
  // q
  bool q_in, q_all;
  closure_status(occ, qxi ? iqx - 1 : iqx, iqx, qyi ? iqy - 1 : iqy, iqy, q_in, q_all);
  close_piece();
  if (q_in && !q_all && !pv_left_in) {
    n_points++;
    best_point = fminf(best_point, dist_f32(qx, qy));
  }

  ScanOut o;
  if (n_lines > 0 && n_points > 0) {
    o.kind = SCAN_COLLECTION;
    o.dist = norm_f32(__fsub_rn(fqx, fpx), __fsub_rn(fqy, fpy));
  } else if (n_lines == 1) {
    o.kind = SCAN_LINE;
    const double dx = __dsub_rn(l0x, px), dy = __dsub_rn(l0y, py);
    const double d = __dsub_rn(__dsqrt_rn(__fma_rn(dy, dy, __dmul_rn(dx, dx))), 1e-3);
    o.dist = (float)(d > 0.0 ? d : 0.0);
  } else if (n_lines > 1) {
    o.kind = SCAN_MULTILINE;
    const float d = __fsub_rn(best_line, 0.001f);
    o.dist = d > 0.0f ? d : 0.0f;
  } else if (n_points == 1) {
    o.kind = SCAN_POINT;
    o.dist = 0.0f;
  } else if (n_points > 1) {
    o.kind = SCAN_MULTIPOINT;
    const float d = __fsub_rn(best_point, 0.001f);
    o.dist = d > 0.0f ? d : 0.0f;
  } else {
    o.kind = SCAN_EMPTY;
    o.dist = norm_f32(__fsub_rn(fqx, fpx), __fsub_rn(fqy, fpy));
  }
  return o;
}

// ------------------------------------------------------------------ occupancy accessors
struct OccGlobal {  // bit rows in global memory
  const uint64_t *rows;
  int h, w, wpr;
  APG_DEV bool at(int x, int y) const {
    if ((unsigned)x >= (unsigned)w || (unsigned)y >= (unsigned)h) return false;
    return (rows[y * wpr + (x >> 6)] >> (x & 63)) & 1ULL;
  }
};

struct OccWindow {  // 32-column window rows in LDS; columns [x0, x0+32), rows [y0, y0+nrows)
  const uint32_t *win;
  int x0, y0, nrows;
  APG_DEV bool at(int x, int y) const {
    const unsigned r = (unsigned)(y - y0), c = (unsigned)(x - x0);
    if (r >= (unsigned)nrows || c >= 32u) return false;
    return (win[r] >> c) & 1u;
  }
};

// bits [x0, x0+32) of a bit row (zero outside [0, 64*wpr))
APG_DEV uint32_t extract_window_row(const uint64_t *row, int wpr, int x0) {
  uint32_t res = 0;
  for (int k = 0; k < wpr; k++) {
    const int shift = 64 * k - x0;  // result bit position of row bit 64k
    const uint64_t v = row[k];
    if (shift >= 32 || shift <= -64) continue;
    res |= shift >= 0 ? (uint32_t)(v << shift) : (uint32_t)(v >> (-shift));
  }
  return res;
}

}  // namespace apg
