/*
 * CPU restatement (TEST INFRASTRUCTURE ONLY) of the LIDAR localization hot path:
 *   LIDARLocalization2DEnv.__lidar_scan   ap_gym/envs/lidar_localization2d.py:496-536
 *   LIDARLocalization2DEnv._step          :317-389
 *   LIDARLocalization2DEnv.__get_obs      :238-277   (render-only observation_map skipped)
 *   LIDARLocalization2DEnv.reset          :293-315   + _np_random setter :547-557
 *   TimeLimit.step / _get_time_obs        ap_gym/time_limit.py:113-139
 *   ActivePerceptionEnv.step + normalized MSELossFn   active_perception_env.py:101-121,
 *                                          active_regression_env.py:29-52, loss_fn.py:100-110,261-267
 *   gymnasium SyncVectorEnv NEXT_STEP autoreset (seed+i per sub-env)
 *
 * GEOS semantics (shapely LineString.intersection(union_all(boxes))) are restated per
 * DESIGN.md §LIDAR-scan semantics: parity UNPINNED against real GEOS (absent here); pinned
 * against the exact-rational model in tests/golden/_stubs/shapely through the fixtures.
 *
 * Algorithm here: enumerate every crossing of the segment with the integer grid lines, order the
 * crossings with exact orientation signs (double expansions), classify each crossing/interval
 * against the occupancy grid.  Compiled with -ffp-contract=off (no FMA contraction), matching the
 * reference's evaluation order; explicit fma() only where numpy's OpenBLAS ddot uses one.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "apg_oracle.h"

/* ------------------------------------------------------------ exact orientation sign */
static void two_sum(double a, double b, double *s, double *e) {
  double x = a + b, bv = x - a, av = x - bv;
  *s = x;
  *e = (a - av) + (b - bv);
}

static void two_prod(double a, double b, double *p, double *e) {
  *p = a * b;
  *e = fma(a, b, -*p);
}

/* sign of the exact sum of n doubles (Shewchuk grow-expansion). */
static int exact_sign(const double *terms, int n) {
  double h[64];
  int m = 0;
  for (int i = 0; i < n; i++) {
    double q = terms[i];
    int k = 0;
    for (int j = 0; j < m; j++) {
      double s, e;
      two_sum(q, h[j], &s, &e);
      q = s;
      if (e != 0.0) h[k++] = e;
    }
    if (q != 0.0) h[k++] = q;
    m = k;
  }
  /* nonoverlapping, increasing magnitude: sign of the largest component */
  for (int j = m - 1; j >= 0; j--)
    if (h[j] != 0.0) return h[j] > 0 ? 1 : -1;
  return 0;
}

/* sign of (qx-px)*(vy-py) - (qy-py)*(vx-px), exactly, for double inputs */
static int orient(double px, double py, double qx, double qy, double vx, double vy) {
  double a[2], b[2], c[2], d[2];
  two_sum(qx, -px, &a[0], &a[1]);
  two_sum(vy, -py, &b[0], &b[1]);
  two_sum(qy, -py, &c[0], &c[1]);
  two_sum(vx, -px, &d[0], &d[1]);
  double t[16];
  int n = 0;
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) {
      two_prod(a[i], b[j], &t[n], &t[n + 1]);
      n += 2;
      two_prod(-c[i], d[j], &t[n], &t[n + 1]);
      n += 2;
    }
  return exact_sign(t, n);
}

/* ------------------------------------------------------------ GEOS Intersection::intersection */
static void geos_intersection(double p1x_, double p1y_, double p2x_, double p2y_, double q1x_,
                              double q1y_, double q2x_, double q2y_, double *ox, double *oy) {
  double minX0 = p1x_ < p2x_ ? p1x_ : p2x_, minY0 = p1y_ < p2y_ ? p1y_ : p2y_;
  double maxX0 = p1x_ > p2x_ ? p1x_ : p2x_, maxY0 = p1y_ > p2y_ ? p1y_ : p2y_;
  double minX1 = q1x_ < q2x_ ? q1x_ : q2x_, minY1 = q1y_ < q2y_ ? q1y_ : q2y_;
  double maxX1 = q1x_ > q2x_ ? q1x_ : q2x_, maxY1 = q1y_ > q2y_ ? q1y_ : q2y_;
  double intMinX = minX0 > minX1 ? minX0 : minX1, intMaxX = maxX0 < maxX1 ? maxX0 : maxX1;
  double intMinY = minY0 > minY1 ? minY0 : minY1, intMaxY = maxY0 < maxY1 ? maxY0 : maxY1;
  double midx = (intMinX + intMaxX) / 2.0, midy = (intMinY + intMaxY) / 2.0;
  double p1x = p1x_ - midx, p1y = p1y_ - midy, p2x = p2x_ - midx, p2y = p2y_ - midy;
  double q1x = q1x_ - midx, q1y = q1y_ - midy, q2x = q2x_ - midx, q2y = q2y_ - midy;
  double px = p1y - p2y, py = p2x - p1x, pw = p1x * p2y - p2x * p1y;
  double qx = q1y - q2y, qy = q2x - q1x, qw = q1x * q2y - q2x * q1y;
  double x = py * qw - qy * pw, y = qx * pw - px * qw, w = px * qy - qx * py;
  *ox = x / w + midx;
  *oy = y / w + midy;
}

/* ------------------------------------------------------------ scan */
static inline int occ_at(const uint8_t *map, int h, int w, long cx, long cy) {
  if (cx < 0 || cy < 0 || cx >= w || cy >= h) return 0;
  return map[cy * (long)w + cx] != 0;
}

typedef struct {
  double x, y;  /* node coordinate as GEOS would emit it */
  int node;     /* 1 if the event is a node of the noded line */
  int onb;      /* event lies on the boundary of U */
} scan_event;

/* closure-cell occupancy of a point given the integer cell ranges [i0,i1] x [j0,j1] */
static void cells_status(const uint8_t *map, int h, int w, long i0, long i1, long j0, long j1,
                         int *in_u, int *all_occ) {
  int any = 0, all = 1;
  for (long i = i0; i <= i1; i++)
    for (long j = j0; j <= j1; j++) {
      int o = occ_at(map, h, w, i, j);
      any |= o;
      all &= o;
    }
  *in_u = any;
  *all_occ = all;
}

static float norm_f32(float dx, float dy) {
  float s = dx * dx + dy * dy; /* f32 products, f32 sum (numpy sdot on 2 elements) */
  return (float)sqrt((double)s);
}

float orc_lidar_scan(const uint8_t *map, int h, int w, float fpx, float fpy, float fqx, float fqy,
                     int *kind_out) {
  const double px = fpx, py = fpy, qx = fqx, qy = fqy;
  const double dx = qx - px, dy = qy - py; /* signs only */
  const int sx = dx > 0 ? 1 : (dx < 0 ? -1 : 0), sy = dy > 0 ? 1 : (dy < 0 ? -1 : 0);
  /* crossings strictly inside the segment */
  long ax0, ax1, by0, by1; /* ranges of integer lines crossed, in travel order */
  long nxl = 0, nyl = 0;
  if (sx > 0) {
    ax0 = (long)floor(px) + 1;
    ax1 = (long)ceil(qx) - 1;
  } else if (sx < 0) {
    ax0 = (long)ceil(px) - 1;
    ax1 = (long)floor(qx) + 1;
  } else {
    ax0 = 1;
    ax1 = 0;
  }
  if (sy > 0) {
    by0 = (long)floor(py) + 1;
    by1 = (long)ceil(qy) - 1;
  } else if (sy < 0) {
    by0 = (long)ceil(py) - 1;
    by1 = (long)floor(qy) + 1;
  } else {
    by0 = 1;
    by1 = 0;
  }
  if (sx != 0) nxl = sx > 0 ? (ax1 >= ax0 ? ax1 - ax0 + 1 : 0) : (ax0 >= ax1 ? ax0 - ax1 + 1 : 0);
  if (sy != 0) nyl = sy > 0 ? (by1 >= by0 ? by1 - by0 + 1 : 0) : (by0 >= by1 ? by0 - by1 + 1 : 0);

  int cap = (int)(nxl + nyl + 2);
  scan_event *ev = (scan_event *)malloc(sizeof(scan_event) * (size_t)cap);
  int *ivl_in = (int *)malloc(sizeof(int) * (size_t)cap); /* interval after event k is in U */
  int ne = 0;

  const int colv = (sx == 0 && floor(px) == px); /* collinear with a vertical grid line */
  const int colh = (sy == 0 && floor(py) == py);
  /* cell of the open interval that follows p */
  long cx = sx > 0 ? (long)floor(px) : (sx < 0 ? (long)ceil(px) - 1 : (long)floor(px));
  long cy = sy > 0 ? (long)floor(py) : (sy < 0 ? (long)ceil(py) - 1 : (long)floor(py));

#define IVL_IN(CX, CY)                                                                  \
  (colv ? (occ_at(map, h, w, (CX)-1, (CY)) | occ_at(map, h, w, (CX), (CY)))             \
        : colh ? (occ_at(map, h, w, (CX), (CY)-1) | occ_at(map, h, w, (CX), (CY)))      \
               : occ_at(map, h, w, (CX), (CY)))

  /* event 0: p */
  {
    long i1 = (long)floor(px), j1 = (long)floor(py);
    long i0 = floor(px) == px ? i1 - 1 : i1, j0 = floor(py) == py ? j1 - 1 : j1;
    int in_u, all;
    cells_status(map, h, w, i0, i1, j0, j1, &in_u, &all);
    ev[0].x = px;
    ev[0].y = py;
    ev[0].node = 1;
    ev[0].onb = in_u && !all;
    ivl_in[0] = IVL_IN(colv ? (long)px : cx, colh ? (long)py : cy);
    ne = 1;
  }
  long xi = 0, yi = 0;
  while (xi < nxl || yi < nyl) {
    long a = ax0 + sx * xi, b = by0 + sy * yi;
    int takex, takey;
    if (xi < nxl && yi < nyl) {
      /* sign(t_a - t_b) = -sign(orient(p,q,(a,b))) * sx * sy */
      int o = orient(px, py, qx, qy, (double)a, (double)b);
      int c = -o * sx * sy;
      takex = c <= 0;
      takey = c >= 0;
    } else {
      takex = xi < nxl;
      takey = !takex;
    }
    scan_event *e = &ev[ne];
    long i0, i1, j0, j1;
    if (takex && takey) { /* lattice point */
      i0 = a - 1;
      i1 = a;
      j0 = b - 1;
      j1 = b;
      e->x = (double)a;
      e->y = (double)b;
    } else if (takex) {
      i0 = a - 1;
      i1 = a;
      j0 = j1 = colh ? 0 : cy;
      if (colh) {
        j0 = (long)py - 1;
        j1 = (long)py;
      }
      geos_intersection(px, py, qx, qy, (double)a, (double)cy, (double)a, (double)(cy + 1), &e->x,
                        &e->y);
    } else {
      j0 = b - 1;
      j1 = b;
      i0 = i1 = cx;
      if (colv) {
        i0 = (long)px - 1;
        i1 = (long)px;
      }
      geos_intersection(px, py, qx, qy, (double)cx, (double)b, (double)(cx + 1), (double)b, &e->x,
                        &e->y);
    }
    if (colv || colh) { /* collinear: every crossing is a lattice point */
      e->x = colv ? px : (double)a;
      e->y = colh ? py : (double)b;
    }
    int in_u, all;
    cells_status(map, h, w, i0, i1, j0, j1, &in_u, &all);
    e->onb = in_u && !all;
    e->node = e->onb;
    if (takex) {
      cx += sx;
      xi++;
    }
    if (takey) {
      cy += sy;
      yi++;
    }
    ivl_in[ne] = IVL_IN(colv ? (long)px : cx, colh ? (long)py : cy);
    ne++;
  }
  /* event last: q */
  {
    long i1 = (long)floor(qx), j1 = (long)floor(qy);
    long i0 = floor(qx) == qx ? i1 - 1 : i1, j0 = floor(qy) == qy ? j1 - 1 : j1;
    int in_u, all;
    cells_status(map, h, w, i0, i1, j0, j1, &in_u, &all);
    ev[ne].x = qx;
    ev[ne].y = qy;
    ev[ne].node = 1;
    ev[ne].onb = in_u && !all;
    ivl_in[ne] = 0;
    ne++;
  }
#undef IVL_IN

  /* walk nodes: pieces between consecutive nodes */
  int n_lines = 0, n_points = 0;
  double first_x = 0, first_y = 0;                /* start of the single line piece */
  float best_line = INFINITY, best_point = INFINITY; /* f32 distances for Multi* */
  int prev_node = 0, prev_piece_in = 0;
  for (int k = 1; k < ne; k++) {
    if (!ev[k].node) continue;
    int piece_in = ivl_in[prev_node]; /* constant between nodes */
    if (piece_in) {
      n_lines++;
      if (n_lines == 1) {
        first_x = ev[prev_node].x;
        first_y = ev[prev_node].y;
      }
      float fx = (float)ev[prev_node].x - fpx, fy = (float)ev[prev_node].y - fpy;
      float dd = norm_f32(fx, fy);
      if (dd < best_line) best_line = dd;
    }
    /* isolated point at prev_node? (needs both neighbouring pieces outside U) */
    if (ev[prev_node].onb && !piece_in && !(prev_node > 0 && prev_piece_in)) {
      n_points++;
      float fx = (float)ev[prev_node].x - fpx, fy = (float)ev[prev_node].y - fpy;
      float dd = norm_f32(fx, fy);
      if (dd < best_point) best_point = dd;
    }
    prev_piece_in = piece_in;
    prev_node = k;
  }
  /* the final node (q) */
  if (ev[prev_node].onb && !prev_piece_in) {
    n_points++;
    float fx = (float)ev[prev_node].x - fpx, fy = (float)ev[prev_node].y - fpy;
    float dd = norm_f32(fx, fy);
    if (dd < best_point) best_point = dd;
  }
  free(ev);
  free(ivl_in);

  int kind;
  float dist;
  if (n_lines > 0 && n_points > 0) {
    kind = ORC_COLLECTION;
    dist = norm_f32(fqx - fpx, fqy - fpy);
  } else if (n_lines == 1) {
    kind = ORC_LINESTRING;
    double ddx = first_x - px, ddy = first_y - py;
    double d = sqrt(fma(ddy, ddy, ddx * ddx)) - 1e-3; /* numpy f64 norm: OpenBLAS ddot w/ FMA */
    dist = (float)(d > 0.0 ? d : 0.0);
  } else if (n_lines > 1) {
    kind = ORC_MULTILINESTRING;
    float d = best_line - 0.001f;
    dist = d > 0.0f ? d : 0.0f;
  } else if (n_points == 1) {
    kind = ORC_POINT;
    dist = 0.0f;
  } else if (n_points > 1) {
    kind = ORC_MULTIPOINT;
    float d = best_point - 0.001f;
    dist = d > 0.0f ? d : 0.0f;
  } else {
    kind = ORC_EMPTY;
    dist = norm_f32(fqx - fpx, fqy - fpy);
  }
  if (kind_out) *kind_out = kind;
  return dist;
}

/* ------------------------------------------------------------ vectorised env */
struct orc_lidar_env {
  int n, kind, h, w, is_static, beams, step_limit;
  int max_rooms, door_width; /* FloorMapDatasetRooms parameters of the dynamic maps (default 10, 3) */
  const uint8_t *pool;       /* kind 2: the dataset's maps [pool_len][h][w] (borrowed), any FloorMapDataset */
  int64_t pool_len;
  orc_map_fn map_fn;         /* kind 2 without a pool: get_data_point(idx) called at every draw (any len) */
  void *map_ctx;
  float range;
  float *dirs;        /* [beams][2] scaled beam vectors (lidar_directions) */
  orc_pcg64 *rng;     /* env np_random */
  orc_pcg64 *it_rng;  /* DatasetIterator rng (dynamic maps) */
  uint8_t *maps;      /* [n or 1][h][w] */
  uint64_t *map_idx;
  float *pos, *init_pos;
  int32_t *elapsed;
  uint8_t *first_step; /* pos/initial_pos still alias the same ndarray (reset :305) */
  uint8_t *autoreset;
  int no_free; /* a map without free cells was drawn (sticky) */
};

orc_lidar_env *orc_lidar_create(int num_envs, int map_kind, int h, int w, int static_map,
                                int static_map_index, int beams, float lidar_range, int step_limit,
                                const float *beam_dirs) {
  orc_lidar_env *e = (orc_lidar_env *)calloc(1, sizeof(*e));
  e->n = num_envs;
  e->kind = map_kind;
  e->h = h;
  e->w = w;
  e->is_static = static_map;
  e->beams = beams;
  e->range = lidar_range;
  e->step_limit = step_limit;
  e->max_rooms = 10;
  e->door_width = 3;
  e->dirs = (float *)malloc(sizeof(float) * 2 * beams);
  memcpy(e->dirs, beam_dirs, sizeof(float) * 2 * beams);
  e->rng = (orc_pcg64 *)calloc(num_envs, sizeof(orc_pcg64));
  e->it_rng = (orc_pcg64 *)calloc(num_envs, sizeof(orc_pcg64));
  e->maps = (uint8_t *)calloc((size_t)(static_map ? 1 : num_envs) * h * w, 1);
  e->map_idx = (uint64_t *)calloc(num_envs, sizeof(uint64_t));
  e->pos = (float *)calloc(2 * num_envs, sizeof(float));
  e->init_pos = (float *)calloc(2 * num_envs, sizeof(float));
  e->elapsed = (int32_t *)calloc(num_envs, sizeof(int32_t));
  e->first_step = (uint8_t *)calloc(num_envs, 1);
  e->autoreset = (uint8_t *)calloc(num_envs, 1);
  if (static_map && map_kind != 2) {
    int r = map_kind == 0 ? orc_rooms_map((uint64_t)static_map_index, h, w, 10, 3, e->maps)
                          : orc_maze_map((uint64_t)static_map_index, h, w, 1.0, e->maps);
    if (r != 0) {
      orc_lidar_destroy(e);
      return NULL;
    }
  }
  if (static_map)
    for (int i = 0; i < num_envs; i++) e->map_idx[i] = (uint64_t)static_map_index;
  return e;
}

void orc_lidar_destroy(orc_lidar_env *e) {
  if (!e) return;
  free(e->dirs);
  free(e->rng);
  free(e->it_rng);
  free(e->maps);
  free(e->map_idx);
  free(e->pos);
  free(e->init_pos);
  free(e->elapsed);
  free(e->first_step);
  free(e->autoreset);
  free(e);
}

static const uint8_t *env_map(const orc_lidar_env *e, int i) {
  return e->maps + (e->is_static ? 0 : (size_t)i * e->h * e->w);
}

static void write_obs(orc_lidar_env *e, int i, float *lidar, float *odometry, float *time_step,
                      float *map_obs) {
  const uint8_t *m = env_map(e, i);
  float px = e->pos[2 * i], py = e->pos[2 * i + 1];
  for (int b = 0; b < e->beams; b++) {
    float qx = px + e->dirs[2 * b], qy = py + e->dirs[2 * b + 1];
    float d = orc_lidar_scan(m, e->h, e->w, px, py, qx, qy, NULL);
    float v = d / e->range;
    lidar[(size_t)i * e->beams + b] = v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
  }
  /* odometry_norm = (odo - (-max)) / (max - (-max)) * 2 - 1  (lidar_localization2d.py:263-270) */
  float mx = (float)e->w, my = (float)e->h;
  float ox = px - e->init_pos[2 * i], oy = py - e->init_pos[2 * i + 1];
  odometry[2 * i] = (ox - (-mx)) / (mx - (-mx)) * 2.0f - 1.0f;
  odometry[2 * i + 1] = (oy - (-my)) / (my - (-my)) * 2.0f - 1.0f;
  time_step[i] = (float)(2.0 * e->elapsed[i] / e->step_limit - 1.0);
  if (map_obs && !e->is_static) {
    float *mo = map_obs + (size_t)i * e->h * e->w;
    for (int k = 0; k < e->h * e->w; k++) mo[k] = (float)m[k] / 255.0f;
  }
}

static void env_reset_one(orc_lidar_env *e, int i) {
  if (!e->is_static && e->kind == 2) {
    /* DatasetIterator.__next__ (dataset_iterator.py:26-32): idx = rng.integers(0, len(dataset)), then
       dataset.get_data_point(idx) -- the pool's map idx */
    uint64_t idx = (uint64_t)orc_integers(&e->it_rng[i], 0, e->pool_len);
    uint8_t *m = e->maps + (size_t)i * e->h * e->w;
    if (e->map_fn) {
      if (e->map_fn(e->map_ctx, idx, m) != 0) e->no_free = 1; /* (the callback failed: flagged like a bad map) */
    } else {
      memcpy(m, e->pool + (size_t)idx * e->h * e->w, (size_t)e->h * e->w);
    }
    e->map_idx[i] = idx;
  } else if (!e->is_static) {
    uint64_t idx = (uint64_t)orc_next32(&e->it_rng[i]); /* integers(0, 2**32) */
    uint8_t *m = e->maps + (size_t)i * e->h * e->w;
    if (e->kind == 0)
      orc_rooms_map(idx, e->h, e->w, e->max_rooms, e->door_width, m);
    else
      orc_maze_map(idx, e->h, e->w, 1.0, m);
    e->map_idx[i] = idx;
  }
  const uint8_t *m = env_map(e, i);
  int64_t nfree = 0;
  for (int k = 0; k < e->h * e->w; k++) nfree += m[k] == 0;
  if (nfree == 0) { /* numpy raises ValueError("high <= 0") (lidar_localization2d.py:302-303) */
    e->no_free = 1;
    e->pos[2 * i] = e->pos[2 * i + 1] = 0.5f;
    e->init_pos[2 * i] = e->init_pos[2 * i + 1] = 0.5f;
    e->first_step[i] = 1;
    e->elapsed[i] = 0;
    return;
  }
  int64_t pick = orc_integers(&e->rng[i], 0, nfree);
  int64_t c = -1;
  for (int k = 0; k < e->h * e->w; k++) {
    if (m[k] == 0 && ++c == pick) {
      e->pos[2 * i] = (float)(k % e->w) + 0.5f;
      e->pos[2 * i + 1] = (float)(k / e->w) + 0.5f;
      break;
    }
  }
  e->init_pos[2 * i] = e->pos[2 * i];
  e->init_pos[2 * i + 1] = e->pos[2 * i + 1];
  e->first_step[i] = 1;
  e->elapsed[i] = 0;
}

void orc_lidar_reset(orc_lidar_env *e, uint64_t seed, float *lidar, float *odometry,
                     float *time_step, float *map_obs, uint64_t *map_idx) {
  for (int i = 0; i < e->n; i++) {
    orc_seed(seed + (uint64_t)i, &e->rng[i]);
    if (!e->is_static) orc_seed(orc_integers_u32_endpoint(&e->rng[i]), &e->it_rng[i]);
    env_reset_one(e, i);
    e->autoreset[i] = 0;
    write_obs(e, i, lidar, odometry, time_step, map_obs);
    if (map_idx) map_idx[i] = e->map_idx[i];
  }
}

/* One sub-env's SyncVectorEnv step (NEXT_STEP autoreset, TimeLimit, LIDARLocalization2DEnv.step);
   sub-envs touch only their own state and output rows.  Returns the NaN error bits. */
static int step_one(orc_lidar_env *e, int i, const float *action, const float *prediction, float *lidar,
                    float *odometry, float *time_step, float *map_obs, double *reward, uint8_t *terminated,
                    uint8_t *truncated, float *base_reward, float *target, float *loss, uint8_t *info_mask,
                    uint64_t *map_idx) {
  int err = 0;
  {
    if (e->autoreset[i]) {
      env_reset_one(e, i);
      write_obs(e, i, lidar, odometry, time_step, map_obs);
      reward[i] = 0.0;
      terminated[i] = truncated[i] = 0;
      base_reward[i] = 0.0f;
      target[2 * i] = target[2 * i + 1] = 0.0f;
      loss[i] = 0.0f;
      info_mask[i] = 0;
      if (map_idx) map_idx[i] = e->map_idx[i];
      e->autoreset[i] = 0;
      return 0;
    }
    const uint8_t *m = env_map(e, i);
    float ax = action[2 * i], ay = action[2 * i + 1];
    float prx = prediction[2 * i], pry = prediction[2 * i + 1];
    if (isnan(ax) || isnan(ay)) err |= 1;
    if (isnan(prx) || isnan(pry)) err |= 2;
    float *pos = &e->pos[2 * i];
    float mapw = (float)e->w, maph = (float)e->h;
    float lpx = pos[0], lpy = pos[1];
    float br = 0.1f - 0.001f * (ax * ax + ay * ay);
    float mag = norm_f32(ax, ay);
    if (mag > 1.0f) {
      ax = ax / mag;
      ay = ay / mag;
    }
    float tx = pos[0] + ax, ty = pos[1] + ay;
    float dirx = tx - pos[0], diry = ty - pos[1];
    float total = norm_f32(dirx, diry);
    if (total > 0.0f) {
      dirx /= total;
      diry /= total;
      float d = orc_lidar_scan(m, e->h, e->w, pos[0], pos[1], tx, ty, NULL);
      pos[0] = pos[0] + dirx * d;
      pos[1] = pos[1] + diry * d;
      float rem = total - d;
      if (rem > 1e-5f) {
        float rvx = dirx * rem, rvy = diry * rem;
        float kept[2];
        int nk = 0;
        if (rvx > 1e-5f) kept[nk++] = rvx;
        if (rvy > 1e-5f) kept[nk++] = rvy;
        if (nk > 0) {
          float c0x = nk == 2 ? kept[0] : kept[0], c0y = 0.0f;
          float c1x = 0.0f, c1y = nk == 2 ? kept[1] : kept[0];
          float d0 = orc_lidar_scan(m, e->h, e->w, pos[0], pos[1], pos[0] + c0x, pos[1] + c0y, NULL);
          float d1 = orc_lidar_scan(m, e->h, e->w, pos[0], pos[1], pos[0] + c1x, pos[1] + c1y, NULL);
          float cx, cy, dd;
          if (d0 > 0.0f) {
            cx = c0x;
            cy = c0y;
            dd = d0;
          } else {
            cx = c1x;
            cy = c1y;
            dd = d1;
          }
          float nrm = norm_f32(cx, cy);
          pos[0] = pos[0] + cx / nrm * dd;
          pos[1] = pos[1] + cy / nrm * dd;
        }
      }
    }
    if (e->first_step[i]) { /* initial_pos is the same ndarray as pos until np.clip rebinds pos */
      e->init_pos[2 * i] = pos[0];
      e->init_pos[2 * i + 1] = pos[1];
      e->first_step[i] = 0;
    }
    int term = 0;
    if (pos[0] < 0.0f || pos[1] < 0.0f || pos[0] >= mapw || pos[1] >= maph) term = 1;
    pos[0] = pos[0] < 0.0f ? 0.0f : (pos[0] > mapw ? mapw : pos[0]);
    pos[1] = pos[1] < 0.0f ? 0.0f : (pos[1] > maph ? maph : pos[1]);
    float tgx = lpx / mapw * 2.0f - 1.0f, tgy = lpy / maph * 2.0f - 1.0f;
    e->elapsed[i] += 1;
    if (e->elapsed[i] >= e->step_limit) term = 1;
    write_obs(e, i, lidar, odometry, time_step, map_obs);
    /* normalized MSE: mean((pred - target)^2) * f32(scale) + f32(-0.0), scale = 1/(4/12) */
    float ex = prx - tgx, ey = pry - tgy;
    float mse = (ex * ex + ey * ey) / 2.0f;
    float l = mse * 3.0f + (-0.0f);
    base_reward[i] = br;
    target[2 * i] = tgx;
    target[2 * i + 1] = tgy;
    loss[i] = l;
    reward[i] = (double)(br - l);
    terminated[i] = (uint8_t)term;
    truncated[i] = 0;
    info_mask[i] = 1;
    if (map_idx) map_idx[i] = e->map_idx[i];
    e->autoreset[i] = (uint8_t)term;
  }
  return err;
}

int orc_lidar_step(orc_lidar_env *e, const float *action, const float *prediction, float *lidar,
                   float *odometry, float *time_step, float *map_obs, double *reward,
                   uint8_t *terminated, uint8_t *truncated, float *base_reward, float *target,
                   float *loss, uint8_t *info_mask, uint64_t *map_idx) {
  int err = 0;
  for (int i = 0; i < e->n; i++)
    err |= step_one(e, i, action, prediction, lidar, odometry, time_step, map_obs, reward, terminated, truncated,
                    base_reward, target, loss, info_mask, map_idx);
  return err;
}

/* The same step with the sub-envs spread over `threads` OpenMP threads (bench.py's multi-core CPU
   baseline row); outputs are identical to orc_lidar_step's. */
int orc_lidar_step_mt(orc_lidar_env *e, int threads, const float *action, const float *prediction, float *lidar,
                      float *odometry, float *time_step, float *map_obs, double *reward, uint8_t *terminated,
                      uint8_t *truncated, float *base_reward, float *target, float *loss, uint8_t *info_mask,
                      uint64_t *map_idx) {
  int err = 0;
#pragma omp parallel for num_threads(threads) reduction(| : err) schedule(dynamic, 64)
  for (int i = 0; i < e->n; i++)
    err |= step_one(e, i, action, prediction, lidar, odometry, time_step, map_obs, reward, terminated, truncated,
                    base_reward, target, loss, info_mask, map_idx);
  return err;
}

void orc_lidar_get_state(const orc_lidar_env *e, float *pos, float *init_pos, int32_t *elapsed,
                         uint8_t *autoreset) {
  if (pos) memcpy(pos, e->pos, sizeof(float) * 2 * e->n);
  if (init_pos) memcpy(init_pos, e->init_pos, sizeof(float) * 2 * e->n);
  if (elapsed) memcpy(elapsed, e->elapsed, sizeof(int32_t) * e->n);
  if (autoreset) memcpy(autoreset, e->autoreset, e->n);
}

/* FloorMapDatasetRooms(max_rooms=..., door_width=...) for the dynamic maps of later resets */
void orc_lidar_set_rooms(orc_lidar_env *e, int max_rooms, int door_width) {
  e->max_rooms = max_rooms;
  e->door_width = door_width;
}

/* kind 2 (any finite FloorMapDataset): its maps [pool_len][h][w] (0/1 bytes, borrowed: the caller keeps them alive).
   Static envs take pool map static_map_index (lidar_localization2d.py:177-178). */
int orc_lidar_set_pool(orc_lidar_env *e, const uint8_t *maps, int64_t pool_len, int static_map_index) {
  if (e->kind != 2 || pool_len < 1) return -1;
  e->pool = maps;
  e->pool_len = pool_len;
  if (e->is_static) {
    if (static_map_index < 0 || static_map_index >= pool_len) return -1;
    memcpy(e->maps, maps + (size_t)static_map_index * e->h * e->w, (size_t)e->h * e->w);
  }
  return 0;
}

/* kind 2, dynamic maps, fetched per draw: fn(ctx, idx, out[h][w] 0/1 bytes) is the dataset's get_data_point(idx)
   (dataset_iterator.py:26-32), called at every reset with idx = integers(0, len) of the env's DatasetIterator stream.
   Any len >= 1 (e.g. 2**32). */
int orc_lidar_set_map_source(orc_lidar_env *e, orc_map_fn fn, void *ctx, int64_t len) {
  if (e->kind != 2 || e->is_static || !fn || len < 1) return -1;
  e->map_fn = fn;
  e->map_ctx = ctx;
  e->pool = NULL;
  e->pool_len = len;
  return 0;
}

/* 1 once a map without a free cell was drawn (the reference raised ValueError there) */
int orc_lidar_no_free(const orc_lidar_env *e) { return e->no_free; }
