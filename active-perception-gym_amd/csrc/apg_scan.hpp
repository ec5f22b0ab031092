// apg_scan.hpp — exact LIDAR segment scan on device (one lane = one segment).
//
// Replaces LIDARLocalization2DEnv.__lidar_scan (ap_gym/envs/lidar_localization2d.py:496-536), i.e.
// shapely.LineString([p, q]).intersection(union_all(unit boxes)) followed by the reference's
// branch on the GEOS result type.  Semantics: the segment is noded at every
// boundary point of the closed union U it meets (edge crossings, boundary lattice vertices); noded
// pieces inside U are LineStrings, boundary nodes with no adjacent inside piece are Points; the
// result type decides the distance:
//   empty -> |q-p| (f32)         LineString -> max(|c-p|_f64 - 1e-3, 0)    Point -> 0
//   Multi* -> max(min_i |f32(c_i)-p|_f32 - 1e-3f, 0)                    mixed -> |q-p| (f32)
//
// Algorithm: a DDA walk over grid-line crossings in segment order.  The loop body is branch-free
// except for node bookkeeping: the crossing order comes from the exact orientation predicate
// (filter, exact fallback only on near-ties), and the closure cells of each crossing are read as
// a 2x2 bit quad from two occupancy row words (`rows.row(y)` = cells [x0, x0 + width) of map row y, zero
// outside the map; Rows::word = uint32_t for the LDS window of the step kernel, uint64_t for rows read from
// global memory, so a segment may span width - 3 columns).  GEOS's crossing coordinate is computed only for nodes that start a
// line piece.
#pragma once
#include "apg_device.hpp"

namespace apg {

enum : int { SCAN_EMPTY = 0, SCAN_LINE = 1, SCAN_MULTILINE = 2, SCAN_POINT = 3, SCAN_MULTIPOINT = 4,
             SCAN_COLLECTION = 5 };

struct ScanOut {
  float dist;
  int kind;
};

// The reference's `contact_point` of a hit (render path only, lidar_localization2d.py:506-525): the
// LineString entry node in float64, the nearest Multi* node in float32, p for a Point.
struct ScanContact {
  double x, y;
  bool is_f32;
};

// closure quad of cells [i0, i0+di] x [j0, j0+dj] (di, dj in {0, 1}); returns bit0 = any, bit1 = all
template <class Rows>
APG_DEV unsigned quad_status(const Rows &rows, int i0, int di, int j0, int dj) {
  const unsigned m = di ? 3u : 1u;
  const int sh = i0 - rows.x0;
  const unsigned b0 = (unsigned)(rows.row(j0) >> sh) & m;
  const unsigned b1 = (unsigned)(rows.row(j0 + dj) >> sh) & m;
  return ((b0 | b1) != 0u ? 1u : 0u) | ((b0 == m && b1 == m) ? 2u : 0u);
}

// Cheap conservative pre-test: can any occupied cell's closed box meet the segment?  Every closed
// unit box [i, i+1] x [j, j+1] meeting the segment meets its bounding box, i.e. has
// i in [ceil(min x) - 1, floor(max x)] and j in [ceil(min y) - 1, floor(max y)].  When none of those
// cells is occupied the intersection is empty and the scan is SCAN_EMPTY with |q - p| (exactly what
// the walk below returns for it).  Rows/columns are read through the same window as the walk.
// hmax: an upper bound of the box height j1 - j0 + 1 that is uniform across the wave (beams of one
// direction), so row reads past every lane's box are skipped
template <class Rows>
APG_DEV bool scan_may_hit(const Rows &rows, float fpx, float fpy, float fqx, float fqy, int hmax = 8) {
  const int i0 = (int)ceilf(fminf(fpx, fqx)) - 1, i1 = (int)floorf(fmaxf(fpx, fqx));
  const int j0 = (int)ceilf(fminf(fpy, fqy)) - 1, j1 = (int)floorf(fmaxf(fpy, fqy));
  using W = typename Rows::word;
  const int wdt = i1 - i0 + 1;  // <= lidar range + 2 < the word width
  const W mask = ((W(1) << wdt) - W(1)) << (i0 - rows.x0);
  return (rows.or_rows(j0, j1, hmax) & mask) != W(0);
}

APG_DEV ScanOut scan_empty(float fpx, float fpy, float fqx, float fqy) {
  ScanOut o;
  o.kind = SCAN_EMPTY;
  o.dist = norm_f32(__fsub_rn(fqx, fpx), __fsub_rn(fqy, fpy));
  return o;
}

// Result of a walk without lattice crossings from its runs of occupied cells (see lidar_scan_fast):
// n_runs runs, whether the first / last visited cell is occupied, and the crossed edge (from lattice
// point (na, nb), vertical when n_x) where the first run starts unless it starts at p.  Endpoints on a
// grid line can be Point pieces.  One f64 square root serves every outcome.
template <class Rows>
APG_DEV ScanOut scan_runs_result(const Rows &rows, float fpx, float fpy, float fqx, float fqy, int n_runs, bool cur0,
                                 bool cur_last, bool n_x, int na, int nb) {
  const float flpx = floorf(fpx), flpy = floorf(fpy), flqx = floorf(fqx), flqy = floorf(fqy);
  const bool pxi = flpx == fpx, pyi = flpy == fpy, qxi = flqx == fqx, qyi = flqy == fqy;
  // endpoints on the boundary next to an outside interval are Point pieces
  int n_points = 0;
  if ((pxi || pyi) && !cur0 &&
      quad_status(rows, (int)flpx - (pxi ? 1 : 0), pxi ? 1 : 0, (int)flpy - (pyi ? 1 : 0), pyi ? 1 : 0) == 1u)
    n_points++;
  if ((qxi || qyi) && !cur_last &&
      quad_status(rows, (int)flqx - (qxi ? 1 : 0), qxi ? 1 : 0, (int)flqy - (qyi ? 1 : 0), qyi ? 1 : 0) == 1u)
    n_points++;
  const bool hit = n_runs > 0 && n_points == 0;  // LINE / MULTILINE
  double x = fpx, y = fpy;
  if (hit && !cur0)
    geos_intersection((double)fpx, (double)fpy, (double)fqx, (double)fqy, (double)na, (double)nb,
                      (double)(n_x ? na : na + 1), (double)(n_x ? nb + 1 : nb), x, y);
  // LINE: |c - p| in f64; MULTILINE: |f32(c) - p| in f32; EMPTY / COLLECTION: |q - p| in f32
  const bool line = hit && n_runs == 1;
  double arg;
  if (line) {
    const double dx = __dsub_rn(x, (double)fpx), dy = __dsub_rn(y, (double)fpy);
    arg = __fma_rn(dy, dy, __dmul_rn(dx, dx));
  } else {
    const float ex = hit ? __fsub_rn((float)x, fpx) : __fsub_rn(fqx, fpx);
    const float ey = hit ? __fsub_rn((float)y, fpy) : __fsub_rn(fqy, fpy);
    arg = (double)__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
  }
  const double r = __dsqrt_rn(arg);
  ScanOut o;
  if (line) {
    o.kind = SCAN_LINE;
    const double d = __dsub_rn(r, 1e-3);
    o.dist = (float)(d > 0.0 ? d : 0.0);
  } else if (hit) {
    o.kind = SCAN_MULTILINE;
    const float d = __fsub_rn((float)r, 0.001f);
    o.dist = d > 0.0f ? d : 0.0f;
  } else if (n_runs > 0) {
    o.kind = SCAN_COLLECTION;  // lines and points: the reference's `else` branch (no hit)
    o.dist = (float)r;
  } else if (n_points > 0) {
    o.kind = n_points == 1 ? SCAN_POINT : SCAN_MULTIPOINT;
    o.dist = 0.0f;  // POINT: 0; MULTIPOINT: max(min(|p - p|, ...) - 1e-3, 0), p being the first point
  } else {
    o.kind = SCAN_EMPTY;
    o.dist = (float)r;
  }
  return o;
}

// Fast path of the walk when no crossing passes through a lattice point and the segment does not run
// along a grid line.  Then every crossing is an edge crossing between the two cells before and after
// it, so a crossing is a boundary node iff those cells differ, and the pieces are decided by the
// sequence of visited cells: its runs of occupied cells are the line pieces, and the only possible
// Point pieces are p and q themselves (an endpoint on the boundary whose adjacent interval is
// outside; only endpoints on a grid line can be on the boundary).  Lines and points: the reference's
// mixed-collection branch (|q - p|); one run: SCAN_LINE from its start; two or more: SCAN_MULTILINE,
// whose minimum over the runs' f32 start distances is the first run's (any later run start lies >= 1
// further along the ray: between two run starts lie an exit and so three distinct grid lines, two of
// them parallel and one cell apart, which dwarfs the < 1e-4 rounding of the f32 distances); points
// only: SCAN_POINT / SCAN_MULTIPOINT at distance 0 (the first point is p when p is one).  Returns false
// (the caller runs the general walk) when a crossing turns out to be a lattice point or the segment is
// collinear with a grid line; the exact orientation decides near-ties as in the general walk.
#ifndef APG_WALK_INC
#define APG_WALK_INC 0  // 1: crossing order from the incrementally updated f64 orientation (A/B: noise-level, not kept)
#endif
// APG_WALK_INC: the orientation of the next lattice point, O(a, b) = (px - a)(qy - b) - (py - b)(qx - a), is affine
// in (a, b): O(a + sx, b) = O + sx (py - qy), O(a, b + sy) = O + sy (qx - px).  The walk keeps it in f64 and adds one
// increment per crossing.  Error bound: coordinates lie in [0, 512] and segments are < 64 long, so every |O| and
// partial product stays below 2^13 and each f64 operation errs by < 2^-40; the initial value (five operations) plus
// at most 128 increments (each also carrying the < 2^-47 rounding of its increment) stay below 2^-32 in all.  A
// magnitude above ORDER_EPS = 2^-30 therefore has the exact sign; below it the exact predicate decides, as the f32
// filter's undecided band did.
constexpr double ORDER_EPS = 0x1p-30;

template <class W>
struct FastWalk {
  float px, py, qx, qy, sxy;
  int sx, sy, ux, vy, sd, force, a, b, xoff, left;
  W r_c, r_o, r_p;
  bool cur0, cur, bail;
  int n_runs, n_x, na, nb;
#if APG_WALK_INC
  double O, DA, DB;  // orientation of lattice point (a, b) (times sx * sy), its increments for a += sx / b += sy
#endif

  // false when the segment runs along a grid line (the general walk's case)
  template <class Rows>
  APG_DEV bool init(const Rows &rows, float fpx, float fpy, float fqx, float fqy) {
    px = fpx, py = fpy, qx = fqx, qy = fqy;
    sx = (fqx > fpx) - (fqx < fpx), sy = (fqy > fpy) - (fqy < fpy);
    const float flpx = floorf(fpx), flpy = floorf(fpy), flqx = floorf(fqx), flqy = floorf(fqy);
    const bool pxi = flpx == fpx, pyi = flpy == fpy, qxi = flqx == fqx, qyi = flqy == fqy;
    left = 0;
    bail = (sx == 0 && pxi) || (sy == 0 && pyi);
    const int ipx = (int)flpx, ipy = (int)flpy, iqx = (int)flqx, iqy = (int)flqy;
    // first interval's cell (cx, cy); the next x-line to cross is a = cx + ux (likewise b = cy + vy) and
    // the lines strictly inside the segment number nxl / nyl (q's own grid line is not crossed)
    ux = sx > 0 ? 1 : 0, vy = sy > 0 ? 1 : 0;
    const int cx = (sx < 0 && pxi) ? ipx - 1 : ipx;
    const int cy = (sy < 0 && pyi) ? ipy - 1 : ipy;
    a = cx + ux, b = cy + vy;
    int nxl = sx > 0 ? (qxi ? iqx - 1 : iqx) - a + 1 : (sx < 0 ? a - iqx : 0);
    int nyl = sy > 0 ? (qyi ? iqy - 1 : iqy) - b + 1 : (sy < 0 ? b - iqy : 0);
    nxl = nxl < 0 ? 0 : nxl;
    nyl = nyl < 0 ? 0 : nyl;
    // Which line comes next is the orientation of lattice point (a, b) against the ray p -> q extended
    // past q: once one family is used up, its next line is crossed at or beyond q, after every line of
    // the other family still ahead, so the order test needs no "lines left" bookkeeping (and never ties
    // there: those two crossings are distinct points).  Rays along an axis cross one family only.
    force = sx == 0 ? 1 : (sy == 0 ? -1 : 0);  // > 0: y-lines only, < 0: x-lines only
    sd = sy > 0 ? 1 : -1;
    xoff = ux + rows.x0;  // the current column is a - ux: its bit in a window row is a - xoff
    r_c = rows.row(cy), r_o = rows.row(cy + sd), r_p = rows.row(cy + 2 * sd);
    cur0 = ((unsigned)(r_c >> (cx - rows.x0)) & 1u) != 0u;
    cur = cur0;
    n_runs = cur ? 1 : 0;
    n_x = 0, na = 0, nb = 0;  // the first run's entry crossing: lines (na, nb) ahead of it, x-line or not
    sxy = (float)(sx * sy);
    left = bail ? 0 : nxl + nyl;
#if APG_WALK_INC
    {
      const double dpx = fpx, dpy = fpy, dqx = fqx, dqy = fqy, da = (double)a, db = (double)b, s = (double)(sx * sy);
      O = __dmul_rn(__dsub_rn(__dmul_rn(__dsub_rn(dpx, da), __dsub_rn(dqy, db)),
                              __dmul_rn(__dsub_rn(dpy, db), __dsub_rn(dqx, da))), s);
      DA = __dmul_rn(__dsub_rn(dpy, dqy), (double)(sx * sx * sy));  // sx * (py - qy), times sx * sy
      DB = __dmul_rn(__dsub_rn(dqx, dpx), (double)(sy * sx * sy));  // sy * (qx - px), times sx * sy
    }
#endif
    return !bail;
  }

  // f32 filter of the crossing order at (a, b): < 0 x-line first, > 0 y-line first, 0 undecided
  APG_DEV int order() const {
#if APG_WALK_INC
    return O > ORDER_EPS ? -1 : (O < -ORDER_EPS ? 1 : 0);
#endif
    const float fa = (float)a, fb = (float)b;
    const float dl = __fmul_rn(__fsub_rn(px, fa), __fsub_rn(qy, fb));
    const float dr = __fmul_rn(__fsub_rn(py, fb), __fsub_rn(qx, fa));
    const float dsx = __fmul_rn(__fsub_rn(dl, dr), sxy);
    const float bound = 1.7881398e-7f * __fadd_rn(fabsf(dl), fabsf(dr));
    return dsx > bound ? -1 : (-dsx > bound ? 1 : 0);
  }
  APG_DEV bool undecided(int c) const { return force == 0 && c == 0; }
  // exact order for an undecided filter; 0 (a crossing through a lattice point) hands the segment over
  // to the general walk
  APG_DEV int order_exact() {
    const int c = -orient(px, py, qx, qy, (double)a, (double)b) * sx * sy;
    bail = bail || c == 0;
    return c;
  }

  // one crossing; act = false leaves the result state alone (the pair walk's shorter segment, whose
  // position then runs past q: kWrap keeps its row reads inside the window)
  template <bool kWrap, class Rows>
  APG_DEV void step(const Rows &rows, int c, bool act) {
    const bool takex = force != 0 ? force < 0 : c < 0;
    const int pa = a, pb = b;
    a += takex ? sx : 0;
    b += takex ? 0 : sy;
#if APG_WALK_INC
    O = __dadd_rn(O, takex ? DA : DB);
#endif
    r_c = takex ? r_c : r_o;
    r_o = takex ? r_o : r_p;
    const int ry = b - vy + 2 * sd;  // unchanged after an x-crossing; consumed a crossing later at the earliest
    r_p = kWrap ? rows.row(ry) : rows.row_nw(ry);
    bool in;
    if constexpr (sizeof(W) == 4) in = __builtin_amdgcn_ubfe(r_c, (unsigned)(a - xoff), 1u) != 0u;
    else in = ((unsigned)(r_c >> (a - xoff)) & 1u) != 0u;
    const bool rise = act && in && !cur;
    const bool first = rise && n_runs == 0;
    n_x = first ? (int)takex : n_x;
    na = first ? pa : na;
    nb = first ? pb : nb;
    n_runs += rise ? 1 : 0;
    cur = act ? in : cur;
  }

  template <class Rows>
  APG_DEV ScanOut result(const Rows &rows) const {
    // the crossed edge's lower-left lattice point: x-line na in row nb - vy, or y-line nb in column na - ux
    return scan_runs_result(rows, px, py, qx, qy, n_runs, cur0, cur, n_x, n_x ? na : na - ux, n_x ? nb - vy : nb);
  }
};

template <class Rows>
APG_DEV bool lidar_scan_fast(const Rows &rows, float fpx, float fpy, float fqx, float fqy, ScanOut &o) {
  FastWalk<typename Rows::word> w;
  if (!w.init(rows, fpx, fpy, fqx, fqy)) return false;
  for (int left = w.left; left > 0; left--) {  // single exit: a lattice crossing is checked after the loop
    int c = w.order();
    if (w.undecided(c)) c = w.order_exact();
    w.template step<false>(rows, c, true);
  }
  if (w.bail) return false;
  o = w.result(rows);
  return true;
}

// kContact (render path): also report the reference's contact point in *contact; the hot path
// instantiates kContact = false, which compiles to the distance-only walk.
template <class Rows, bool kContact = false>
APG_DEV ScanOut lidar_scan_general(const Rows &rows, float fpx, float fpy, float fqx, float fqy,
                                   ScanContact *contact = nullptr) {
  const double px = fpx, py = fpy, qx = fqx, qy = fqy;
  const int sx = (fqx > fpx) - (fqx < fpx), sy = (fqy > fpy) - (fqy < fpy);
  const float flpx = floorf(fpx), flpy = floorf(fpy), flqx = floorf(fqx), flqy = floorf(fqy);
  const bool pxi = flpx == fpx, pyi = flpy == fpy, qxi = flqx == fqx, qyi = flqy == fqy;
  const int ipx = (int)flpx, ipy = (int)flpy, iqx = (int)flqx, iqy = (int)flqy;
  // integer lines strictly inside the segment, in travel order: ax, ax+sx, ... (nxl of them)
  int ax = 0, nxl = 0, by = 0, nyl = 0;
  if (sx > 0) {
    ax = ipx + 1;
    nxl = (qxi ? iqx - 1 : iqx) - ax + 1;
  } else if (sx < 0) {
    ax = pxi ? ipx - 1 : ipx;
    nxl = ax - iqx;
  }
  if (sy > 0) {
    by = ipy + 1;
    nyl = (qyi ? iqy - 1 : iqy) - by + 1;
  } else if (sy < 0) {
    by = pyi ? ipy - 1 : ipy;
    nyl = by - iqy;
  }
  nxl = nxl < 0 ? 0 : nxl;
  nyl = nyl < 0 ? 0 : nyl;
  // collinear with a grid line: every crossing is a lattice point, intervals touch two cells
  const bool colv = sx == 0 && pxi, colh = sy == 0 && pyi;
  int cx = (sx < 0 && pxi) ? ipx - 1 : ipx;  // cell of the open interval after p
  int cy = (sy < 0 && pyi) ? ipy - 1 : ipy;
  const int ivdi = colv ? 1 : 0, ivdj = colh ? 1 : 0;  // interval cells [cx - ivdi, cx] x [cy - ivdj, cy]

  // node descriptors: type 0 = p, 1 = lattice (a, b), 2 = x-crossing on edge (a, b)-(a, b+1),
  // 3 = y-crossing on edge (a, b)-(a+1, b), 4 = q; packed t | (a + 1024) << 3 | (b + 1024) << 17
  auto pack_node = [](int t, int a, int b) -> uint32_t {
    return (uint32_t)t | ((uint32_t)(a + 1024) << 3) | ((uint32_t)(b + 1024) << 17);
  };
  uint32_t pv = pack_node(0, 0, 0);
  bool pv_onb = quad_status(rows, pxi ? ipx - 1 : ipx, pxi ? 1 : 0, pyi ? ipy - 1 : ipy, pyi ? 1 : 0) == 1u;
  bool pv_left_in = false;
  bool cur_in = quad_status(rows, cx - ivdi, ivdi, cy - ivdj, ivdj) & 1u;
  // The first line start and the first point are resolved after the loop (their coordinates are
  // the only ones the LineString/Point branches need); later ones (Multi* only) are rare and
  // folded into running f32 minima on the spot.
  int n_lines = 0, n_points = 0;
  uint32_t l0 = pv, p0 = pv;
  float later_line = __builtin_inff(), later_point = __builtin_inff();
  float ll_x = 0.0f, ll_y = 0.0f, lp_x = 0.0f, lp_y = 0.0f;  // kContact: f32 nodes of those minima

  auto node_coord = [&](uint32_t node, double &x, double &y) {
    const int t = (int)(node & 7u), a = (int)((node >> 3) & 16383u) - 1024, b = (int)(node >> 17) - 1024;
    if (t == 0) {
      x = px;
      y = py;
    } else if (t == 4) {
      x = qx;
      y = qy;
    } else if (t == 1) {
      x = (double)a;
      y = (double)b;
    } else {
      const bool vert = t == 2;
      geos_intersection(px, py, qx, qy, (double)a, (double)b, (double)(vert ? a : a + 1),
                        (double)(vert ? b + 1 : b), x, y);
    }
  };
  auto dist_f32 = [&](double x, double y) -> float {
    return norm_f32(__fsub_rn((float)x, fpx), __fsub_rn((float)y, fpy));
  };
  // close the piece [previous node, this crossing] (is_line / is_point) and record the crossing as the
  // previous node when it is on the boundary (onb)
  auto close_piece = [&](bool onb, uint32_t node) {
    const bool is_line = onb && cur_in;
    const bool is_point = onb && !cur_in && pv_onb && !pv_left_in;
    if ((is_line && n_lines > 0) || (is_point && n_points > 0)) {  // Multi* only: rare
      double x, y;
      node_coord(pv, x, y);
      const float d = dist_f32(x, y);
      if constexpr (kContact) {  // np.argmin: the first of equal minima
        if (is_line && d < later_line) ll_x = (float)x, ll_y = (float)y;
        if (!is_line && d < later_point) lp_x = (float)x, lp_y = (float)y;
      }
      if (is_line) later_line = fminf(later_line, d);
      else later_point = fminf(later_point, d);
    }
    l0 = (is_line && n_lines == 0) ? pv : l0;
    p0 = (is_point && n_points == 0) ? pv : p0;
    n_lines += is_line ? 1 : 0;
    n_points += is_point ? 1 : 0;
    pv_left_in = onb ? cur_in : pv_left_in;
    pv = onb ? node : pv;
    pv_onb = pv_onb || onb;
  };
  // Every crossing's closure quad lies in rows cy and cy + sd (sd = sign(sy), -1 when sy == 0: the
  // collinear-horizontal quads are rows ipy - 1 = cy - 1 and cy).  They are kept in registers and only
  // shift when a y-crossing moves the walk to the next row; the row after them is read one crossing
  // ahead, so the loop never waits on a just-issued LDS read.
  const int sd = sy > 0 ? 1 : -1;
  using W = typename Rows::word;
  W r_c = rows.row(cy), r_o = rows.row(cy + sd), r_p = rows.row(cy + 2 * sd);
  if (!colv && !colh) {
    // generic segment (not along a grid line): quads are [a-1, a] x cy (x-crossing), cx x [b-1, b]
    // (y-crossing) or the 2 x 2 block at lattice point (a, b); the crossing order is the orientation
    // of (a, b) against p -> q, folded with sign(sx * sy) into one f32 filter
    const float sxy = (float)(sx * sy);
    const unsigned ux = sx > 0 ? 1u : 0u, vy = sy > 0 ? 1u : 0u;  // next cell's offset in the quad
    int a = ax, b = by, rx = nxl, ry = nyl;
    while (rx + ry > 0) {
      const bool hx = rx > 0, hy = ry > 0;
      const float fa = (float)a, fb = (float)b;
      const float dl = __fmul_rn(__fsub_rn(fpx, fa), __fsub_rn(fqy, fb));
      const float dr = __fmul_rn(__fsub_rn(fpy, fb), __fsub_rn(fqx, fa));
      const float dsx = __fmul_rn(__fsub_rn(dl, dr), sxy);  // orientation * sx * sy (exact sign flip)
      const float bound = 1.7881398e-7f * __fadd_rn(fabsf(dl), fabsf(dr));
      int c = dsx > bound ? -1 : (-dsx > bound ? 1 : 0);  // c < 0: x-crossing first, > 0: y first, 0: both
      if (hx && hy && c == 0) c = -orient(fpx, fpy, fqx, fqy, (double)a, (double)b) * sx * sy;  // near-tie
      c = (hx && hy) ? c : (hx ? -1 : 1);
      const bool takex = c <= 0, takey = c >= 0;
      const int i0 = takex ? a - 1 : cx;
      const int sh = i0 - rows.x0;
      const W r0 = (takey && sy < 0) ? r_o : r_c;  // rows.row(j0), j0 = takey ? b - 1 : cy
      const W r1 = (takey && sy > 0) ? r_o : r_c;  // rows.row(j0 + dj)
      const unsigned q0 = (unsigned)(r0 >> sh) & 3u, q1 = (unsigned)(r1 >> sh) & 3u, m = takex ? 3u : 1u;
      const bool onb = ((q0 | q1) & m) != 0u && ((q0 & q1 & m) != m);
      // status of the next open interval: cell (ncx, ncy) at offset (u, v) in the quad
      const unsigned u = takex ? ux : 0u, v = takey ? vy : 0u;
      const bool in_after = (((v ? q1 : q0) >> u) & 1u) != 0u;
      close_piece(onb, pack_node((takex && takey) ? 1 : (takex ? 2 : 3), takex ? a : cx, takey ? b : cy));
      cx += takex ? sx : 0;
      cy += takey ? sy : 0;
      a += takex ? sx : 0;
      b += takey ? sy : 0;
      rx -= takex ? 1 : 0;
      ry -= takey ? 1 : 0;
      cur_in = in_after;
      r_c = takey ? r_o : r_c;
      r_o = takey ? r_p : r_o;
      r_p = rows.row(cy + 2 * sd);  // the same row after an x-crossing: no select on the fresh read
    }
  } else {
    // along a grid line (colv / colh): every crossing is a lattice point, intervals touch two cells
    const int ntot = nxl + nyl;
    int xi = 0, yi = 0;
    while (xi + yi < ntot) {
      const int a = ax + sx * xi, b = by + sy * yi;
      const bool hx = xi < nxl, hy = yi < nyl;
      // c < 0: x-crossing first, c > 0: y-crossing first, 0: both (lattice point)
      const int o = orient_lattice(fpx, fpy, fqx, fqy, a, b);
      const int c = (hx && hy) ? -o * sx * sy : (hx ? -1 : 1);
      const bool takex = c <= 0, takey = c >= 0;
      // closure quad of the crossing: cells [i0, i0+di] x [j0, j0+dj]
      const int i0 = takex ? a - 1 : (colv ? ipx - 1 : cx);
      const int j0 = takey ? b - 1 : (colh ? ipy - 1 : cy);
      const bool di = takex || colv;
      const int sh = i0 - rows.x0;
      const W r0 = takey ? (sy > 0 ? r_c : r_o) : (colh ? r_o : r_c);  // rows.row(j0)
      const W r1 = (takey && sy > 0) ? r_o : r_c;                      // rows.row(j0 + dj)
      const unsigned q0 = (unsigned)(r0 >> sh) & 3u, q1 = (unsigned)(r1 >> sh) & 3u, m = di ? 3u : 1u;
      const bool onb = ((q0 | q1) & m) != 0u && ((q0 & q1 & m) != m);
      const int ncx = cx + (takex ? sx : 0), ncy = cy + (takey ? sy : 0);
      // status of the next open interval from the same quad: cell (ncx, ncy) (+ its collinear twin)
      const unsigned u = (unsigned)(ncx - i0), v = (unsigned)(ncy - j0);
      const unsigned rowv = v ? q1 : q0;
      const bool in_after =
          colv ? (rowv & 3u) != 0u : (colh ? (((q0 | q1) >> u) & 1u) != 0u : ((rowv >> u) & 1u) != 0u);
      const bool lattice = (takex && takey) || (takex && colh) || (takey && colv);
      close_piece(onb, pack_node(lattice ? 1 : (takex ? 2 : 3), takex ? a : (colv ? ipx : cx),
                                 takey ? b : (colh ? ipy : cy)));
      cx = ncx;
      cy = ncy;
      xi += takex ? 1 : 0;
      yi += takey ? 1 : 0;
      cur_in = in_after;
      r_c = takey ? r_o : r_c;
      r_o = takey ? r_p : r_o;
      r_p = rows.row(ncy + 2 * sd);
    }
  }
  // q: always a node
  const unsigned qst = quad_status(rows, qxi ? iqx - 1 : iqx, qxi ? 1 : 0, qyi ? iqy - 1 : iqy, qyi ? 1 : 0);
  {  // close the last piece [previous node, q] (predicated like the loop body: no pointer selects)
    const bool is_line = cur_in, is_point = !cur_in && pv_onb && !pv_left_in;
    if ((is_line && n_lines > 0) || (is_point && n_points > 0)) {
      double x, y;
      node_coord(pv, x, y);
      const float d = dist_f32(x, y);
      if constexpr (kContact) {
        if (is_line && d < later_line) ll_x = (float)x, ll_y = (float)y;
        if (!is_line && d < later_point) lp_x = (float)x, lp_y = (float)y;
      }
      if (is_line) later_line = fminf(later_line, d);
      else later_point = fminf(later_point, d);
    }
    l0 = (is_line && n_lines == 0) ? pv : l0;
    p0 = (is_point && n_points == 0) ? pv : p0;
    n_lines += is_line ? 1 : 0;
    n_points += is_point ? 1 : 0;
    pv_left_in = cur_in;
  }
  pv_onb = qst == 1u;
  if (pv_onb && !pv_left_in) {
    if (n_points == 0) {
      p0 = pack_node(4, 0, 0);
    } else {
      const float d = dist_f32(qx, qy);
      if constexpr (kContact) {
        if (d < later_point) lp_x = fqx, lp_y = fqy;
      }
      later_point = fminf(later_point, d);
    }
    n_points++;
  }

  ScanOut o;
  const float full = norm_f32(__fsub_rn(fqx, fpx), __fsub_rn(fqy, fpy));
  o.kind = SCAN_EMPTY;
  o.dist = full;
  if (n_lines > 0 && n_points > 0) {
    o.kind = SCAN_COLLECTION;  // mixed points and lines: the reference's `else` branch (no hit)
  } else if (n_lines > 0) {
    double x, y;
    node_coord(l0, x, y);
    if (n_lines == 1) {
      o.kind = SCAN_LINE;
      const double dx = __dsub_rn(x, px), dy = __dsub_rn(y, py);
      const double d = __dsub_rn(__dsqrt_rn(__fma_rn(dy, dy, __dmul_rn(dx, dx))), 1e-3);
      o.dist = (float)(d > 0.0 ? d : 0.0);
      if constexpr (kContact) *contact = ScanContact{x, y, false};
    } else {
      o.kind = SCAN_MULTILINE;
      const float d0 = dist_f32(x, y);
      const float d = __fsub_rn(fminf(d0, later_line), 0.001f);
      o.dist = d > 0.0f ? d : 0.0f;
      if constexpr (kContact) {
        const bool later = later_line < d0;
        *contact = ScanContact{later ? ll_x : (float)x, later ? ll_y : (float)y, true};
      }
    }
  } else if (n_points == 1) {
    o.kind = SCAN_POINT;
    o.dist = 0.0f;
    if constexpr (kContact) *contact = ScanContact{fpx, fpy, true};
  } else if (n_points > 1) {
    double x, y;
    node_coord(p0, x, y);
    o.kind = SCAN_MULTIPOINT;
    const float d0 = dist_f32(x, y);
    const float d = __fsub_rn(fminf(d0, later_point), 0.001f);
    o.dist = d > 0.0f ? d : 0.0f;
    if constexpr (kContact) {
      const bool later = later_point < d0;
      *contact = ScanContact{later ? lp_x : (float)x, later ? lp_y : (float)y, true};
    }
  }
  return o;
}

template <class Rows, bool kContact = false>
APG_DEV ScanOut lidar_scan_walk(const Rows &rows, float fpx, float fpy, float fqx, float fqy,
                                ScanContact *contact = nullptr) {
  if constexpr (!kContact) {
    ScanOut fo;
    if (lidar_scan_fast(rows, fpx, fpy, fqx, fqy, fo)) return fo;
  }
  return lidar_scan_general<Rows, kContact>(rows, fpx, fpy, fqx, fqy, contact);
}

template <class Rows>
APG_DEV ScanOut lidar_scan(const Rows &rows, float fpx, float fpy, float fqx, float fqy) {
  if (!scan_may_hit(rows, fpx, fpy, fqx, fqy)) return scan_empty(fpx, fpy, fqx, fqy);
  return lidar_scan_walk(rows, fpx, fpy, fqx, fqy);
}

// ------------------------------------------------------------------ occupancy row sources
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

struct RowsWindow {  // 32-row x 32-column window staged in LDS (rows [y0, y0+32)); callers keep
  typedef uint32_t word;
  const uint32_t *win;  // every access inside the window (see k_lidar_step), so no bounds test
  int x0, y0, nrows;
  APG_DEV uint32_t row(int y) const { return win[(unsigned)(y - y0) & 31u]; }
  APG_DEV uint32_t row_nw(int y) const { return win[y - y0]; }  // y known to lie in the window
  // OR of rows [j0, j1] (inside the window): eight loads at immediate offsets from row j0, masked past j1
  // (they may read up to 7 words beyond the window: the LDS layout pads the last one), a loop only for
  // boxes taller than 8 rows
  APG_DEV uint32_t or_rows(int j0, int j1, int hmax) const {
    const uint32_t *w = win + (j0 - y0);
    const int h = j1 - j0 + 1;
    uint32_t acc = 0u;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      if (t >= hmax) break;  // wave-uniform
      const uint32_t v = w[t];
      acc |= t < h ? v : 0u;
    }
    for (int t = 8; t < h; t++) acc |= w[t];
    return acc;
  }
};

// bits [x0, x0+64) of a bit row (zero outside [0, 64*wpr))
APG_DEV uint64_t extract_window_row64(const uint64_t *row, int wpr, int x0) {
  const int q = x0 >> 6, o = x0 & 63;  // floor division: x0 may be negative
  const uint64_t lo = (q >= 0 && q < wpr) ? row[q] : 0ULL, hi = (q + 1 >= 0 && q + 1 < wpr) ? row[q + 1] : 0ULL;
  return (lo >> o) | ((hi << 1) << (63 - o));
}

struct RowsGlobal {  // bit rows in global memory, read through a 64-column window at x0 (segments up to 61 long)
  typedef uint64_t word;
  const uint64_t *occ;
  int h, wpr, x0;
  APG_DEV uint64_t row(int y) const {
    if ((unsigned)y >= (unsigned)h) return 0ULL;
    return extract_window_row64(occ + (size_t)y * wpr, wpr, x0);
  }
  APG_DEV uint64_t row_nw(int y) const { return row(y); }
  APG_DEV uint64_t or_rows(int j0, int j1, int) const {
    uint64_t acc = 0ULL;
    for (int j = j0; j <= j1; j++) acc |= row(j);
    return acc;
  }
};

}  // namespace apg
