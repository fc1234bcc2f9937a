/*
 * pf_oracle.c -- CPU restatement of the reference's fusion path.  TEST INFRASTRUCTURE ONLY:
 * see the header comment of pf_oracle.h ("parity unpinned": the reference is not buildable in
 * this image and ships no golden vectors; this file is the checker the HIP path is tested
 * against, never part of the product).
 *
 * Citations are to /root/reference (Depth.cpp, Main.cpp, ilmbase22/include/ImathVec.h).
 * Compile with -O2 -ffp-contract=off: every float expression below is evaluated in the
 * reference's order with separately rounded multiplies and adds.
 */
#define _GNU_SOURCE
#include "pf_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MYPI PFO_MYPI
#define NAN_MARKER 0x7FBADBADu /* signalling-NaN payload: arithmetic never produces it */

uint32_t pfo_nan_marker(void) { return NAN_MARKER; }

void pfo_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ---------------- Imath Vec3<float> semantics (ImathVec.h) ---------------- */
static inline float v3_dot(const float a[3], const float b[3])
{ /* ImathVec.h:1467-1470: x*v.x + y*v.y + z*v.z, left to right */
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static inline void v3_cross(const float a[3], const float b[3], float o[3])
{ /* ImathVec.h:1481-1486 */
    float x = a[1] * b[2] - a[2] * b[1];
    float y = a[2] * b[0] - a[0] * b[2];
    float z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static float v3_length(const float a[3])
{ /* ImathVec.h:1631-1671 (length + lengthTiny) */
    float l2 = v3_dot(a, a);
    if (l2 < 2.0f * FLT_MIN) {
        float ax = a[0] >= 0.0f ? a[0] : -a[0];
        float ay = a[1] >= 0.0f ? a[1] : -a[1];
        float az = a[2] >= 0.0f ? a[2] : -a[2];
        float mx = ax;
        if (mx < ay) mx = ay;
        if (mx < az) mx = az;
        if (mx == 0.0f) return 0.0f;
        ax /= mx; ay /= mx; az /= mx;
        return mx * sqrtf(ax * ax + ay * ay + az * az);
    }
    return sqrtf(l2);
}
static void v3_normalize(float a[3])
{ /* ImathVec.h:1682-1700: divides by the length (no reciprocal) */
    float l = v3_length(a);
    if (l != 0.0f) { a[0] /= l; a[1] /= l; a[2] /= l; }
}
static float v2_length(float x, float y)
{ /* ImathVec.h:1145-1180 */
    float l2 = x * x + y * y;
    if (l2 < 2.0f * FLT_MIN) {
        float ax = x >= 0.0f ? x : -x, ay = y >= 0.0f ? y : -y;
        float mx = ax;
        if (mx < ay) mx = ay;
        if (mx == 0.0f) return 0.0f;
        ax /= mx; ay /= mx;
        return mx * sqrtf(ax * ax + ay * ay);
    }
    return sqrtf(l2);
}
static inline void v3_add(const float a[3], const float b[3], float o[3])
{ o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2]; }
static inline void v3_sub(const float a[3], const float b[3], float o[3])
{ o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; }
static inline void v3_scale(const float a[3], float s, float o[3])
{ o[0] = a[0] * s; o[1] = a[1] * s; o[2] = a[2] * s; }

/* ---------------- projection ---------------- */
void pfo_sph_to_world(float az, float zen, float out[3])
{ /* Depth.cpp:2955-2958; g++ fuses the sin/cos pairs into sincosf */
    float sz, cz, sa, ca;
    sincosf(zen, &sz, &cz);
    sincosf(az, &sa, &ca);
    out[0] = sz * ca;
    out[1] = sz * sa;
    out[2] = cz;
}

void pfo_world_to_sph(const float pin[3], float out[2])
{ /* Depth.cpp:2960-2971 */
    float p[3] = {pin[0], pin[1], pin[2]};
    v3_normalize(p);
    float az = (float)fmod((double)atan2f(p[1], p[0]), 2 * MYPI);
    if (az < 0) az = (float)((double)az + 2 * MYPI);
    float zen = atan2f(v2_length(p[0], p[1]), p[2]);
    out[0] = az;
    out[1] = zen;
}

void pfo_set_window(pfo_tile* t, float aL, float aR, float zT, float zD)
{ /* Depth.cpp:120-155 */
    t->az_left = aL; t->az_right = aR; t->zen_top = zT; t->zen_down = zD;
    float mid[3];
    pfo_sph_to_world((aL + aR) / 2, (zT + zD) / 2, mid);
    const float zup[3] = {0.0f, 0.0f, 1.0f};
    float left[3], up[3];
    v3_cross(zup, mid, left);
    v3_normalize(left);
    v3_cross(left, mid, up);
    v3_normalize(up);
    float ta = tanf(fabsf(aR - aL) / 2);
    float tz = tanf(fabsf(zT - zD) / 2);
    float s[3], lm[3], rm[3], um[3], dm[3];
    v3_scale(left, ta, s); v3_add(mid, s, lm);
    v3_scale(left, ta, s); v3_sub(mid, s, rm);
    v3_scale(up, tz, s);   v3_sub(mid, s, um);
    v3_scale(up, tz, s);   v3_add(mid, s, dm);
    float a[3], b[3], c[3];
    /* corner = middle + (X_middle - middle) + (Y_middle - middle), left to right */
    v3_sub(lm, mid, a); v3_add(mid, a, c); v3_sub(um, mid, b); v3_add(c, b, t->corner0);
    v3_sub(lm, mid, a); v3_add(mid, a, c); v3_sub(dm, mid, b); v3_add(c, b, t->corner1);
    v3_sub(rm, mid, a); v3_add(mid, a, c); v3_sub(dm, mid, b); v3_add(c, b, t->corner2);
    v3_sub(rm, mid, a); v3_add(mid, a, c); v3_sub(um, mid, b); v3_add(c, b, t->corner3);
    v3_sub(rm, lm, t->hedge);
    v3_sub(dm, um, t->vedge);
    memcpy(t->middle, mid, sizeof(mid));
}

/* SphericalTo2D with the direction's trig already evaluated (dir = (sz*ca, sz*sa, cz)). */
static void sph_to_2d_trig(const pfo_tile* t, float sz, float cz, float ca, float sa,
                           float out[2])
{ /* Depth.cpp:168-182 with LinePlaneIntersection (Depth.cpp:34-42), p = 0, n = p0 = middle */
    float dir[3] = {sz * ca, sz * sa, cz};
    float p0mp[3] = {t->middle[0] - 0.0f, t->middle[1] - 0.0f, t->middle[2] - 0.0f};
    float tt = v3_dot(p0mp, t->middle) / v3_dot(dir, t->middle);
    float pos[3] = {0.0f + tt * dir[0], 0.0f + tt * dir[1], 0.0f + tt * dir[2]};
    float e[3];
    v3_sub(pos, t->corner0, e);
    float hl = v3_length(t->hedge), vl = v3_length(t->vedge);
    out[0] = (v3_dot(e, t->hedge) / hl) / hl;
    out[1] = (v3_dot(e, t->vedge) / vl) / vl;
}

void pfo_sph_to_2d(const pfo_tile* t, float az, float zen, float out[2])
{
    float sz, cz, sa, ca;
    sincosf(zen, &sz, &cz);
    sincosf(az, &sa, &ca);
    sph_to_2d_trig(t, sz, cz, ca, sa, out);
}

void pfo_to_spherical_coord(const pfo_tile* t, float x, float y, float out[2])
{ /* Depth.cpp:157-166: corner0 + hedge*x + vedge*y, then WorldToSpherical */
    float a[3], b[3], pos[3];
    v3_scale(t->hedge, x, a);
    v3_add(t->corner0, a, pos);
    v3_scale(t->vedge, y, b);
    v3_add(pos, b, pos);
    pfo_world_to_sph(pos, out);
}

long long pfo_tile_index(const pfo_tile* t, float x, float y)
{ /* Depth.cpp:111-118 */
    int X = (int)(x * (float)(t->width - 1));
    int Y = (int)(y * (float)(t->height - 1));
    return ((long long)Y * t->width + X) * t->channels;
}

static inline long long clamp_index(const pfo_tile* t, long long idx, long long* oob)
{
    long long n = (long long)t->width * t->height * t->channels;
    if (idx < 0 || idx >= n) {
        if (oob) (*oob)++;
        idx = idx < 0 ? 0 : n - t->channels;
    }
    return idx;
}

float pfo_tile_value(const pfo_tile* t, const float* tiles, float x, float y)
{
    long long idx = clamp_index(t, pfo_tile_index(t, x, y), NULL);
    return tiles[t->offset + idx];
}

float pfo_emap_value_at_coord(const float* emap, int w, int h, int c, float az, float zen)
{ /* Depth.cpp:551-556: promoted to double through MYPI, truncated */
    int x = (int)((double)az / (MYPI * 2) * (double)(float)(w - 1));
    int y = (int)((double)zen / MYPI * (double)(float)(h - 1));
    return emap[((long long)y * w + x) * c];
}

float pfo_grid_azimuth(int xx, int w)
{ /* Depth.cpp:1591: (float)xx / (float)(w-1) * 2 * MYPI, stored in a Vec2f */
    return (float)((double)((float)xx / (float)(w - 1) * 2.0f) * MYPI);
}
float pfo_grid_zenith(int yy, int h)
{
    return (float)((double)((float)yy / (float)(h - 1)) * MYPI);
}

/* ---------------- registration ---------------- */
int pfo_reg_grid(const pfo_tile* t, float zr0, float zr1, int* cols, int* rows, float* zt,
                 float* zd)
{ /* Depth.cpp:1267-1304 */
    const float subd = (float)(1 / 180.0 * MYPI); /* D2R(1) stored as float */
    *cols = (int)roundf(fabsf(t->ranges[1] - t->ranges[0]) / subd);
    float top = zr0 > t->ranges[2] ? zr0 : t->ranges[2]; /* MAX2 */
    float down = zr1 < t->ranges[3] ? zr1 : t->ranges[3]; /* MIN2 */
    *rows = (int)roundf(fabsf(down - top) / subd);
    *zt = top;
    *zd = down;
    return (*cols + 1) * (*rows + 1);
}

static inline double clamp_depth(double v)
{ /* Depth.cpp:1353-1364 */
    if (v < 1e-4) v = 1e-4;
    else if (v > (1 - 1e-4)) v = 1 - 1e-4;
    return v;
}

int pfo_reg_samples(const pfo_tile* t, const float* tiles, const float* emap, int ew, int eh,
                    int ec, float zr0, float zr1, double* xs, double* ys)
{ /* Depth.cpp:1328-1387 */
    int cols, rows;
    float zt, zd;
    pfo_reg_grid(t, zr0, zr1, &cols, &rows, &zt, &zd);
    int k = 0;
    for (int r = 0; r <= rows; r++) {
        for (int c = 0; c <= cols; c++) {
            float cx = t->ranges[0] + (t->ranges[1] - t->ranges[0]) * (float)c / (float)cols;
            float cy = zt + (zd - zt) * (float)r / (float)rows;
            float xy[2];
            pfo_sph_to_2d(t, cx, cy, xy);
            if (xy[0] < 0) xy[0] = 0;
            if (xy[0] > 1) xy[0] = 1;
            if (xy[1] < 0) xy[1] = 0;
            if (xy[1] > 1) xy[1] = 1;
            double d0 = clamp_depth((double)pfo_tile_value(t, tiles, xy[0], xy[1]));
            double d1 = clamp_depth((double)pfo_emap_value_at_coord(emap, ew, eh, ec, cx, cy));
            xs[k] = d0;
            ys[k] = d1;
            k++;
        }
    }
    return k;
}

#define REG_LANES 256
#define REG_NSUM 15

/* Jacobian row J = (X3, X2, X, 1) of FunctorDepth2Depth3 (Depth.cpp:1124-1130, Weight = 1):
 * X2 = x*x, X3 = x*x*x.  The 15 sums are the upper triangle of J^T J, J^T y and y^T y. */
static inline void reg_terms(double x, double y, double o[REG_NSUM])
{
    double X = x, X2 = x * x, X3 = x * x * x;
    o[0] = X3 * X3; o[1] = X3 * X2; o[2] = X3 * X; o[3] = X3;
    o[4] = X2 * X2; o[5] = X2 * X;  o[6] = X2;
    o[7] = X * X;   o[8] = X;       o[9] = 1.0;
    o[10] = X3 * y; o[11] = X2 * y; o[12] = X * y; o[13] = y;
    o[14] = y * y;
}

/* Solve the (deg+1)x(deg+1) normal equations by partially pivoted Gaussian elimination.
 * Returns 0, or -1 when a pivot vanishes (rank deficient). */
static int solve_normal(const double S[REG_NSUM], int degree, double* coef)
{
    /* basis index b in 0..3 <-> power (3-b); pick the trailing (degree+1) powers */
    static const int idx[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
    int n = degree + 1, off = 3 - degree;
    double A[4][5];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) A[i][j] = S[idx[i + off][j + off]];
        A[i][n] = S[10 + i + off];
    }
    for (int k = 0; k < n; k++) {
        int piv = k;
        double best = fabs(A[k][k]);
        for (int i = k + 1; i < n; i++)
            if (fabs(A[i][k]) > best) { best = fabs(A[i][k]); piv = i; }
        if (!(best > 0.0)) return -1;
        if (piv != k)
            for (int j = 0; j <= n; j++) { double tmp = A[k][j]; A[k][j] = A[piv][j]; A[piv][j] = tmp; }
        for (int i = k + 1; i < n; i++) {
            double f = A[i][k] / A[k][k];
            for (int j = k; j <= n; j++) A[i][j] = A[i][j] - f * A[k][j];
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = A[i][n];
        for (int j = i + 1; j < n; j++) s = s - A[i][j] * coef[j];
        coef[i] = s / A[i][i];
    }
    return 0;
}

int pfo_register_tile(const pfo_tile* t, const float* tiles, const float* emap, int ew, int eh,
                      int ec, float zr0, float zr1, int degree, double* coef64, float* abcd)
{
    return pfo_register_tile_solver(t, tiles, emap, ew, eh, ec, zr0, zr1, degree,
                                    PFO_SOLVER_NORMAL, coef64, abcd);
}

int pfo_register_tile_solver(const pfo_tile* t, const float* tiles, const float* emap, int ew,
                             int eh, int ec, float zr0, float zr1, int degree, int solver,
                             double* coef64, float* abcd)
{
    int cols, rows;
    float zt, zd;
    int ns = pfo_reg_grid(t, zr0, zr1, &cols, &rows, &zt, &zd);
    if (cols <= 0 || rows <= 0 || degree < 0 || degree > 3) return -1;
    double* xs = (double*)malloc(sizeof(double) * ns);
    double* ys = (double*)malloc(sizeof(double) * ns);
    pfo_reg_samples(t, tiles, emap, ew, eh, ec, zr0, zr1, xs, ys);
    /* lane l accumulates samples l, l+256, ... sequentially; then a pairwise tree over lanes */
    double part[REG_LANES][REG_NSUM];
    memset(part, 0, sizeof(part));
    for (int l = 0; l < REG_LANES; l++)
        for (int s = l; s < ns; s += REG_LANES) {
            double o[REG_NSUM];
            reg_terms(xs[s], ys[s], o);
            for (int k = 0; k < REG_NSUM; k++) part[l][k] = part[l][k] + o[k];
        }
    for (int stride = REG_LANES / 2; stride >= 1; stride /= 2)
        for (int l = 0; l < stride; l++)
            for (int k = 0; k < REG_NSUM; k++) part[l][k] = part[l][k] + part[l + stride][k];
    free(xs);
    free(ys);
    if (solver == PFO_SOLVER_LM && degree == 3) {
        /* the reference's solver: Ceres LM from (1,1,1,1), in the moment form (pf_oracle_lm.c) */
        double c[4];
        pfo_lm_moments(part[0], c, NULL);
        for (int i = 0; i < 4; i++) {
            if (coef64) coef64[i] = c[i];
            abcd[i] = (float)c[i];
        }
        return 3;
    }
    double coef[4] = {0, 0, 0, 0};
    int d = degree, rc = -1;
    while (d >= 0 && (rc = solve_normal(part[0], d, coef)) != 0) d--; /* rank-deficient fallback */
    if (rc != 0) { coef[0] = 0.0; d = 0; }
    double full[4] = {0, 0, 0, 0};
    for (int i = 0; i <= d; i++) full[3 - d + i] = coef[i];
    for (int i = 0; i < 4; i++) {
        if (coef64) coef64[i] = full[i];
        abcd[i] = (float)full[i];
    }
    return d;
}

void pfo_depth_to_depth(const pfo_tile* t, float* tiles, const float abcd[4])
{ /* Depth.cpp:245-274 */
    float a = abcd[0], b = abcd[1], c = abcd[2], d = abcd[3];
    float* data = tiles + t->offset;
    for (int y = 0; y < t->height; y++)
        for (int x = 0; x < t->width; x++) {
            long long i = ((long long)y * t->width + x) * t->channels;
            float X = data[i];
            if (X < 1e-4) X = (float)1e-4;
            else if (X > (1 - 1e-4)) X = (float)(1 - 1e-4);
            float Y = a * X * X * X + b * X * X + c * X + d;
            if (Y < 0) Y = 0;
            else if (Y > 1) Y = 1;
            data[i] = Y;
        }
}

/* ---------------- fusion ---------------- */
int pfo_level_dims(int out_w, int out_h, float zr0, float zr1, int level, pfo_level* L)
{ /* Depth.cpp:1420-1437, 1650-1675 */
    int max_level = out_w >= 4096 ? 4 : 3;
    if (level < 0 || level >= max_level) return -1;
    L->max_level = max_level;
    L->w = (int)(out_w / pow(2, max_level - 1 - level));
    L->h = (int)(out_h / pow(2, max_level - 1 - level));
    L->h0 = (int)floor((double)((float)L->h * zr0) / MYPI);
    L->h1 = (int)ceil((double)((float)L->h * zr1) / MYPI);
    static const int it3[3] = {200, 100, 50};
    static const int it4[4] = {200, 150, 100, 50};
    L->iters = max_level == 3 ? it3[level] : it4[level];
    return 0;
}

void pfo_seed_level0(const float* emap, int ew, int eh, int ec, const pfo_level* L, float* buf)
{ /* Depth.cpp:1442-1465 */
    int w = L->w, h = L->h;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            if (y < L->h0 || y > L->h1) buf[(long long)y * w + x] = 0;
            else
                buf[(long long)y * w + x] = pfo_emap_value_at_coord(
                    emap, ew, eh, ec, pfo_grid_azimuth(x, w), pfo_grid_zenith(y, h));
        }
}

void pfo_upsample(const float* prev, const pfo_level* L, float* buf)
{ /* Depth.cpp:1467-1485 */
    int w = L->w, h = L->h, wp = w / 2;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) buf[(long long)y * w + x] = prev[(long long)(y / 2) * wp + x / 2];
}

int pfo_tile_box(const pfo_tile* t, const pfo_level* L, int* px0, int* px1, int* py0, int* py1,
                 int* pxs)
{ /* Depth.cpp:1497-1562 (enlargement disabled at :1522, :1543, clamps kept) */
    int w = L->w, h = L->h;
    int x0 = (int)round((double)t->ranges[0] / (2 * MYPI) * (double)(w - 1));
    int x1 = (int)round((double)t->ranges[1] / (2 * MYPI) * (double)(w - 1));
    int y0 = (int)round((double)t->ranges[2] / MYPI * (double)(h - 1));
    int y1 = (int)round((double)t->ranges[3] / MYPI * (double)(h - 1));
    int xs = x1 >= x0 ? 1 : -1;
    if (x0 < 0) x0 = 0;
    if (x0 >= w) x0 = w - 1;
    if (x1 < 0) x1 = 0;
    if (x1 >= w) x1 = w - 1;
    if (y0 < 0) y0 = 0;
    if (y0 >= h) y0 = h - 1;
    if (y1 < 0) y1 = 0;
    if (y1 >= h) y1 = h - 1;
    if (y0 <= L->h0) y0 = L->h0 + 1;
    if (y1 >= L->h1) y1 = L->h1 - 1;
    *px0 = x0; *px1 = x1; *py0 = y0; *py1 = y1; *pxs = xs;
    return x0 == x1 ? -1 : 0;
}

/* Laplacian target of one tile at pixel (X, Y): the std::map order of the 5-point mask is
 * (X-1,Y), (X,Y-1), (X,Y), (X,Y+1), (X+1,Y) (Depth.cpp:1574-1606). */
static float target_one(const pfo_tile* t, const float* tile_data, const pfo_level* L, int X,
                        int Y, long long* oops, long long* oob)
{
    static const int dx[5] = {-1, 0, 0, 0, 1}, dy[5] = {0, -1, 0, 1, 0};
    static const float wt[5] = {-0.25f, -0.25f, 1.0f, -0.25f, -0.25f};
    float Lp = 0;
    for (int k = 0; k < 5; k++) {
        int xx = X + dx[k], yy = Y + dy[k];
        float xy[2];
        pfo_sph_to_2d(t, pfo_grid_azimuth(xx, L->w), pfo_grid_zenith(yy, L->h), xy);
        if (xy[0] < 0 || xy[0] > 1 || xy[1] < 0 || xy[1] > 1) (*oops)++;
        long long idx = clamp_index(t, pfo_tile_index(t, xy[0], xy[1]), oob);
        float val = tile_data[t->offset + idx];
        Lp += val * wt[k];
    }
    return Lp;
}

int pfo_targets(const pfo_tile* tiles, int ntiles, const float* tile_data, const pfo_level* L,
                float* Lsum, int32_t* n, long long* oops_out, long long* oob_out)
{ /* Depth.cpp:1487-1624.  Returns -1 for a degenerate box, -2 when a pixel is covered by more
   * than 40 tiles (normalised stencil weights stop being exactly {1,-0.25}: see pfo_jacobi). */
    int w = L->w, h = L->h;
    memset(Lsum, 0, sizeof(float) * (size_t)w * h);
    memset(n, 0, sizeof(int32_t) * (size_t)w * h);
    long long oops = 0, oob = 0;
    for (int p = 0; p < ntiles; p++) {
        int x0, x1, y0, y1, xs;
        if (pfo_tile_box(&tiles[p], L, &x0, &x1, &y0, &y1, &xs) != 0) return -1;
    }
    /* tile order = the reference's single-thread order; bit-identical to any thread count for
     * coverage <= 2 (float addition is commutative) */
    for (int p = 0; p < ntiles; p++) {
        int x0, x1, y0, y1, xs;
        pfo_tile_box(&tiles[p], L, &x0, &x1, &y0, &y1, &xs);
        int X = x0;
        while (1) { /* X from x0 up to, but excluding, x1 (Depth.cpp:1565-1623) */
            long long lo = 0, lb = 0;
#pragma omp parallel for schedule(static) reduction(+ : lo, lb)
            for (int Y = y0; Y <= y1; Y++) {
                float Lp = target_one(&tiles[p], tile_data, L, X, Y, &lo, &lb);
                Lsum[(long long)Y * w + X] += Lp;
                n[(long long)Y * w + X] += 1;
            }
            oops += lo;
            oob += lb;
            X += xs;
            if (X == x1) break;
        }
    }
    for (long long i = 0; i < (long long)w * h; i++)
        if (n[i] > 40) return -2;
    if (oops_out) *oops_out = oops;
    if (oob_out) *oob_out = oob;
    return 0;
}

static inline float bits_to_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t float_to_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

void pfo_normalize(const float* Lsum, const int32_t* n, const pfo_level* L, float* Lnorm)
{ /* Depth.cpp:1626-1647: scale = mask_center(1) / center(n) applied when n not in {0,1} */
    int w = L->w, h = L->h;
    const float marker = bits_to_float(NAN_MARKER);
    for (long long i = 0; i < (long long)w * h; i++) {
        int Y = (int)(i / w);
        if (Y <= L->h0 || Y >= L->h1 || n[i] == 0) { Lnorm[i] = marker; continue; }
        float Lv = Lsum[i];
        if (n[i] != 1) {
            float center = 0;
            for (int k = 0; k < n[i]; k++) center += 1.0f;
            float scale = 1.0f / center;
            Lv *= scale;
        }
        Lnorm[i] = Lv;
    }
}

void pfo_jacobi(float* buf, float* tmp, const float* Lnorm, const pfo_level* L, int iters)
{ /* Depth.cpp:1649-1718.  Windows with coverage n <= 40 normalise back to exactly
   * {1, -0.25 x4}; the taps are read by linear index, so the east tap of column w-1 is
   * pixel (0, Y+1) exactly as buffer[yy*width + xx] reads it. */
    const int w = L->w;
    const float step_size = 0.5f;
    const float reg = (float)1e-4;
    const float reg_ = 1 - reg;
    const long long beg = (long long)L->h0 * w, end = (long long)(L->h1 + 1) * w;
    const long long npx = (long long)w * L->h;
    for (int it = 0; it < iters; it++) {
        memcpy(tmp, buf, sizeof(float) * npx);
#pragma omp parallel for schedule(static)
        for (long long i = beg; i < end; i++) {
            float Lt = Lnorm[i];
            float cur = 0;
            float tgt;
            if (float_to_bits(Lt) == NAN_MARKER) {
                tgt = 0;
                cur = 0; /* empty window (or the zero-weight centre inserted at :1637) */
            } else {
                tgt = Lt;
                cur += buf[i - 1] * -0.25f;
                cur += buf[i - w] * -0.25f;
                cur += buf[i] * 1.0f;
                cur += buf[i + w] * -0.25f;
                cur += buf[i + 1] * -0.25f;
            }
            float b = buf[i];
            float target_val = b + (tgt - cur) * step_size;
            float v = target_val * reg_ + b * reg;
            if (v < 0) v = 0;
            else if (v > 1) v = 1;
            tmp[i] = v;
        }
        memcpy(buf, tmp, sizeof(float) * npx);
    }
}

void pfo_quantize(const float* buf, int n, uint16_t* out)
{ /* Depth.cpp:1721-1736 */
    for (int i = 0; i < n; i++) {
        float v = buf[i];
        if (v < 0) v = 0;
        if (v > 1) v = 1;
        out[i] = (uint16_t)(v * 65535.0f);
    }
}

int pfo_solve_depth_all(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles,
                        int ntiles, const float* tile_data, int out_w, int out_h, float zr0,
                        float zr1, uint16_t* out, long long* oops_total)
{
    pfo_level L;
    pfo_level_dims(out_w, out_h, zr0, zr1, 0, &L);
    int max_level = L.max_level;
    float* prev = NULL;
    long long oops_all = 0;
    for (int level = 0; level < max_level; level++) {
        pfo_level_dims(out_w, out_h, zr0, zr1, level, &L);
        size_t np = (size_t)L.w * L.h;
        float* buf = (float*)malloc(sizeof(float) * np);
        float* tmp = (float*)malloc(sizeof(float) * np);
        float* Lsum = (float*)malloc(sizeof(float) * np);
        float* Lnorm = (float*)malloc(sizeof(float) * np);
        int32_t* n = (int32_t*)malloc(sizeof(int32_t) * np);
        if (level == 0) pfo_seed_level0(emap, ew, eh, ec, &L, buf);
        else { pfo_upsample(prev, &L, buf); free(prev); prev = NULL; }
        long long oops = 0;
        if (pfo_targets(tiles, ntiles, tile_data, &L, Lsum, n, &oops, NULL) != 0) {
            free(buf); free(tmp); free(Lsum); free(Lnorm); free(n);
            return -1;
        }
        oops_all += oops;
        pfo_normalize(Lsum, n, &L, Lnorm);
        pfo_jacobi(buf, tmp, Lnorm, &L, L.iters);
        free(tmp); free(Lsum); free(Lnorm); free(n);
        if (level == max_level - 1) {
            pfo_quantize(buf, (int)np, out);
            free(buf);
        } else prev = buf;
    }
    if (oops_total) *oops_total = oops_all;
    return 0;
}

int pfo_merge(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles, int ntiles,
              float* tile_data, int out_w, float zr0, float zr1, int degree, int solver,
              uint16_t* out, float* abcd_out)
{ /* Depth.cpp:789-913 */
    for (int p = 0; p < ntiles; p++) {
        float abcd[4];
        if (pfo_register_tile_solver(&tiles[p], tile_data, emap, ew, eh, ec, zr0, zr1, degree,
                                     solver, NULL, abcd) < 0)
            return -2;
        pfo_depth_to_depth(&tiles[p], tile_data, abcd);
        if (abcd_out) memcpy(abcd_out + 4 * p, abcd, sizeof(abcd));
    }
    return pfo_solve_depth_all(emap, ew, eh, ec, tiles, ntiles, tile_data, out_w, out_w / 2,
                               zr0, zr1, out, NULL);
}

/* ---------------- warps ---------------- */
static inline uint32_t mix32(uint32_t x)
{ /* lowbias32 finaliser */
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

uint32_t pfo_hash32(uint32_t seed, uint32_t idx)
{ /* counter-based noise keyed by (seed, pixel).  seed is unique per (panorama, tile) -- the host
   * folds the layout-wide tile index into it (pf_synth.responses), so a shard's sub-layout warps
   * the same noise as the whole layout.  The pixel hash mix32(idx) does not depend on the
   * panorama and the key mix32(seed) does not depend on the pixel; per (panorama, pixel) they
   * meet in one 24x24-bit multiply, the top 24 bits of its low word are the draw. */
    uint32_t x = mix32(idx) ^ mix32(seed);
    return (x & 0xFFFFFFu) * 0x9E3779u;
}

static inline float response(const pfo_response* r, uint32_t idx, float d)
{
    float u = (float)(pfo_hash32(r->seed, idx) >> 8) * (1.0f / 16777216.0f);
    float nz = u * 2.0f - 1.0f;
    float v = r->alpha * d;
    v = v + (r->kappa * d) * d;
    v = v + r->beta;
    v = v + r->sigma * nz;
    if (v < 0) v = 0;
    else if (v > 1) v = 1;
    return v;
}

/* a5's coordinate map of tile pixel (X,Y): (X/(W-1), Y/(H-1)) -> ToSphericalCoord
 * (Depth.cpp:157-166, WorldToSpherical :2960-2971 with glibc atan2f) -> ValueAtCoord's pixel
 * convention (az/2pi*(pw-1), zen/pi*(ph-1)) -> bilinear corner (x0, y0) and weights (fx, fy). */
static inline void warp_coord(const pfo_tile* t, int X, int Y, int pw, int ph, int* x0o, int* y0o,
                              float* fxo, float* fyo)
{
    float xy_x = (float)X / (float)(t->width - 1);
    float xy_y = (float)Y / (float)(t->height - 1);
    float sc[2];
    pfo_to_spherical_coord(t, xy_x, xy_y, sc);
    float px = (float)((double)sc[0] / (2 * MYPI) * (double)(pw - 1));
    float py = (float)((double)sc[1] / MYPI * (double)(ph - 1));
    int x0 = (int)floorf(px), y0 = (int)floorf(py);
    float fx = px - (float)x0, fy = py - (float)y0;
    if (x0 < 0) { x0 = 0; fx = 0; }
    if (y0 < 0) { y0 = 0; fy = 0; }
    if (x0 > pw - 1) { x0 = pw - 1; fx = 0; }
    if (y0 > ph - 1) { y0 = ph - 1; fy = 0; }
    *x0o = x0; *y0o = y0; *fxo = fx; *fyo = fy;
}

void pfo_warp_coords(const pfo_tile* t, int pw, int ph, uint32_t* wxy, float* wfxy)
{ /* the map of one tile: wxy = x0 | y0 << 16, wfxy = (fx, fy) per pixel, row-major */
#pragma omp parallel for schedule(static)
    for (int Y = 0; Y < t->height; Y++)
        for (int X = 0; X < t->width; X++) {
            int x0, y0;
            float fx, fy;
            warp_coord(t, X, Y, pw, ph, &x0, &y0, &fx, &fy);
            long long i = (long long)Y * t->width + X;
            wxy[i] = (uint32_t)x0 | ((uint32_t)y0 << 16);
            wfxy[2 * i] = fx;
            wfxy[2 * i + 1] = fy;
        }
}

void pfo_warp_depth(const float* pano, int pw, int ph, const pfo_tile* tiles, int ntiles,
                    const pfo_response* resp, float* tile_data)
{ /* a5: bilinear sample of the equirectangular map at warp_coord's corner and weights */
    for (int p = 0; p < ntiles; p++) {
        const pfo_tile* t = &tiles[p];
#pragma omp parallel for schedule(static)
        for (int Y = 0; Y < t->height; Y++)
            for (int X = 0; X < t->width; X++) {
                int x0, y0;
                float fx, fy;
                warp_coord(t, X, Y, pw, ph, &x0, &y0, &fx, &fy);
                int x1 = x0 + 1 < pw ? x0 + 1 : pw - 1;
                int y1 = y0 + 1 < ph ? y0 + 1 : ph - 1;
                float g00 = pano[(long long)y0 * pw + x0], g01 = pano[(long long)y0 * pw + x1];
                float g10 = pano[(long long)y1 * pw + x0], g11 = pano[(long long)y1 * pw + x1];
                float top = g00 * (1.0f - fx) + g01 * fx;
                float bot = g10 * (1.0f - fx) + g11 * fx;
                float v = top * (1.0f - fy) + bot * fy;
                uint32_t idx = (uint32_t)(Y * t->width + X);
                if (resp) v = response(&resp[p], idx, v);
                tile_data[t->offset + (long long)idx * t->channels] = v;
            }
    }
}

static void warp_rgb_impl(const uint8_t* pano, int pw, int ph, const pfo_tile* tiles, int ntiles,
                          uint8_t* out, uint32_t* taps)
{ /* a18: the GL camera of SaveCubeMap (Main.cpp:242-326; gluLookAt up = z, gluPerspective
   * fovy/aspect), pixel centres, the exact texcoord map of fs_perspective.txt:67-73 that the
   * sphere mesh (SphereMesh.cpp:154-210) approximates, GL_LINEAR + GL_REPEAT (SphereMesh.cpp:74-
   * 77) on the u8 RGB texture, rows flipped to top-first as stbi_flip_vertically_on_write does.
   * Direction and angles are evaluated in double; parity against real OpenGL is unpinned. */
    long long obase = 0, tbase = 0;
    for (int p = 0; p < ntiles; p++) {
        const pfo_tile* t = &tiles[p];
        float s0 = t->az_left, s1 = t->az_right, s2 = t->zen_top, s3 = t->zen_down;
        float azc = (s1 + s0) / 2, zenc = (s3 + s2) / 2;
        float fovx = (float)((s1 - s0) / MYPI * 180.0);
        float fovy = (float)((s3 - s2) / MYPI * 180.0);
        float aspect = (float)(tan(fovx / 180.0 * MYPI / 2) / tan(fovy / 180.0 * MYPI / 2));
        double f[3] = {cos((double)azc) * sin((double)zenc), sin((double)azc) * sin((double)zenc),
                       cos((double)zenc)};
        double fl = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
        f[0] /= fl; f[1] /= fl; f[2] /= fl;
        double s[3] = {f[1], -f[0], 0.0}; /* f x (0,0,1) */
        double sl = sqrt(s[0] * s[0] + s[1] * s[1]);
        s[0] /= sl; s[1] /= sl;
        double u[3] = {s[1] * f[2] - s[2] * f[1], s[2] * f[0] - s[0] * f[2], s[0] * f[1] - s[1] * f[0]};
        double ty = tan((double)fovy / 180.0 * MYPI / 2), tx = ty * (double)aspect;
        int W = t->width, H = t->height;
#pragma omp parallel for schedule(static)
        for (int r = 0; r < H; r++)
            for (int i = 0; i < W; i++) {
                double xn = 2.0 * (i + 0.5) / W - 1.0, yn = 1.0 - 2.0 * (r + 0.5) / H;
                double d[3];
                for (int k = 0; k < 3; k++) d[k] = f[k] + s[k] * (xn * tx) + u[k] * (yn * ty);
                double az = fmod(atan2(d[1], d[0]), 2 * MYPI);
                if (az < 0) az += 2 * MYPI;
                double zen = atan2(sqrt(d[0] * d[0] + d[1] * d[1]), d[2]);
                float uu = (float)(az / (2 * MYPI)), vv = (float)(zen / MYPI);
                float sx = uu * (float)pw - 0.5f, sy = vv * (float)ph - 0.5f;
                int ix = (int)floorf(sx), iy = (int)floorf(sy);
                float ax = sx - (float)ix, ay = sy - (float)iy;
                int ix0 = ((ix % pw) + pw) % pw, ix1 = (((ix + 1) % pw) + pw) % pw;
                int iy0 = ((iy % ph) + ph) % ph, iy1 = (((iy + 1) % ph) + ph) % ph;
                if (taps) { /* pfo_rgb_taps: the map only */
                    uint32_t* tp = taps + 4 * (tbase + (long long)r * W + i);
                    tp[0] = (uint32_t)ix0 | ((uint32_t)iy0 << 16);
                    tp[1] = (uint32_t)ix1 | ((uint32_t)iy1 << 16);
                    memcpy(&tp[2], &ax, 4);
                    memcpy(&tp[3], &ay, 4);
                    continue;
                }
                for (int c = 0; c < 3; c++) {
                    float t00 = pano[((long long)iy0 * pw + ix0) * 3 + c];
                    float t01 = pano[((long long)iy0 * pw + ix1) * 3 + c];
                    float t10 = pano[((long long)iy1 * pw + ix0) * 3 + c];
                    float t11 = pano[((long long)iy1 * pw + ix1) * 3 + c];
                    float top = t00 * (1.0f - ax) + t01 * ax;
                    float bot = t10 * (1.0f - ax) + t11 * ax;
                    float v = top * (1.0f - ay) + bot * ay;
                    int q = (int)floorf(v + 0.5f);
                    if (q < 0) q = 0;
                    if (q > 255) q = 255;
                    out[obase + ((long long)r * W + i) * 3 + c] = (uint8_t)q;
                }
            }
        obase += (long long)W * H * 3;
        tbase += (long long)W * H;
    }
}

void pfo_warp_rgb(const uint8_t* pano, int pw, int ph, const pfo_tile* tiles, int ntiles,
                  uint8_t* out)
{
    warp_rgb_impl(pano, pw, ph, tiles, ntiles, out, NULL);
}

void pfo_rgb_taps(int pw, int ph, const pfo_tile* tiles, int ntiles, uint32_t* taps)
{ /* the map of pfo_warp_rgb: per tile pixel (tiles in order, rows top-first) {ix0 | iy0 << 16,
   * ix1 | iy1 << 16, bits of ax, bits of ay} */
    warp_rgb_impl(NULL, pw, ph, tiles, ntiles, NULL, taps);
}

/* Parity probe: per pixel of a level, the linear tile index of each of the 5 taps of the first
 * covering tile (tile order), -1 where no tile covers (same contract as pf_probe_taps). */
int pfo_probe_taps(const pfo_tile* tiles, int ntiles, const pfo_level* L, int32_t* out)
{
    static const int dx[5] = {-1, 0, 0, 0, 1}, dy[5] = {0, -1, 0, 1, 0};
    int w = L->w, h = L->h;
    for (long long i = 0; i < (long long)w * h * 5; i++) out[i] = -1;
    int* first = (int*)malloc(sizeof(int) * (size_t)w * h);
    for (long long i = 0; i < (long long)w * h; i++) first[i] = -1;
    for (int p = ntiles - 1; p >= 0; p--) {
        int x0, x1, y0, y1, xs;
        if (pfo_tile_box(&tiles[p], L, &x0, &x1, &y0, &y1, &xs) != 0) { free(first); return -1; }
        for (int X = x0; X != x1; X += xs)
            for (int Y = y0; Y <= y1; Y++) first[(long long)Y * w + X] = p;
    }
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)w * h; i++) {
        int p = first[i];
        if (p < 0) continue;
        int Y = (int)(i / w), X = (int)(i % w);
        for (int k = 0; k < 5; k++) {
            float xy[2];
            pfo_sph_to_2d(&tiles[p], pfo_grid_azimuth(X + dx[k], w), pfo_grid_zenith(Y + dy[k], h), xy);
            out[i * 5 + k] = (int32_t)pfo_tile_index(&tiles[p], xy[0], xy[1]);
        }
    }
    free(first);
    return 0;
}


/* ---- accuracy metrics: ErrorData (Depth.cpp:1980-2213) / ErrorEmap (Depth.cpp:2215-2458) ---- */
static int cmp_f32(const void* a, const void* b)
{
    float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

/* One pixel of the compare loops (Depth.cpp:2033-2053 / :2248-2268). */
static int metrics_px(const float* gt, int gw, int gh, int gc, const float* given,
                      const uint16_t* given16, int w, int given_c, float rx, float ry, int x,
                      int y, int abs_skip, int cap, float depth_max, float* v0, float* v1)
{
    int X = (int)((float)x * rx), Y = (int)((float)y * ry);
    if (X > gw - 1) X = gw - 1;
    if (Y > gh - 1) Y = gh - 1;
    float a = gt[((long long)Y * gw + X) * gc];
    float b = given16 ? (float)given16[(long long)y * w + x] / 65535.0f
                      : given[((long long)y * w + x) * given_c];
    if ((abs_skip ? fabsf(a) : a) < 1e-4) return 0;
    if (cap) {
        a = a < depth_max ? a : depth_max;
        b = b < depth_max ? b : depth_max;
    }
    *v0 = a;
    *v1 = b;
    return 1;
}

void pfo_error_metrics(const float* gt, int gw, int gh, int gc, const float* given,
                       const uint16_t* given16, int w, int h, int given_c, float zr0, float zr1,
                       int align_way, int cap_depth, float* out, int* cnt)
{
    int height0 = (int)(zr0 / PFO_MYPI * h), height1 = (int)(zr1 / PFO_MYPI * h);
    float rx = (float)gw / (float)w, ry = (float)gh / (float)h;
    const float to_matterport = 65535.0f / 4000.0f;
    float depth_max = 10.0f / to_matterport;
    float shift = 1.0f, ls_s = 0.0f, ls_o = 0.0f, gt_med = 0.0f, gv_med = 0.0f;
    int abs_skip = given16 ? 0 : 1;
    if (height0 < 0) height0 = 0;
    if (height1 > h - 1) height1 = h - 1;
    if (align_way == 1) {
        long long cap = (long long)(height1 - height0 + 1) * w, n = 0;
        float* g = (float*)malloc(sizeof(float) * (cap > 0 ? cap : 1));
        float* v = (float*)malloc(sizeof(float) * (cap > 0 ? cap : 1));
        for (int y = height0; y <= height1; y++)
            for (int x = 0; x < w; x++) {
                float a, b;
                if (!metrics_px(gt, gw, gh, gc, given, given16, w, given_c, rx, ry, x, y, abs_skip,
                                cap_depth, depth_max, &a, &b))
                    continue;
                g[n] = a;
                v[n] = b;
                n++;
            }
        qsort(g, n, sizeof(float), cmp_f32);
        qsort(v, n, sizeof(float), cmp_f32);
        if (n > 0) {
            gt_med = g[n / 2];
            gv_med = v[n / 2];
        }
        shift = gt_med / gv_med;
        free(g);
        free(v);
    } else if (align_way == 2) {
        float a00 = 0, a01 = 0, a11 = 0, b0 = 0, b1 = 0;
        for (int y = height0; y <= height1; y++)
            for (int x = 0; x < w; x++) {
                float a, b;
                if (!metrics_px(gt, gw, gh, gc, given, given16, w, given_c, rx, ry, x, y, 0,
                                cap_depth, depth_max, &a, &b))
                    continue;
                a00 += b * b;
                a01 += b;
                a11 += 1;
                b0 += a * b;
                b1 += a;
            }
        float det = a00 * a11 - a01 * a01;
        ls_s = (a11 * b0 - a01 * b1) / det;
        ls_o = (-a01 * b0 + a00 * b1) / det;
    }
    float mse = 0, mae = 0, mre = 0, mselog = 0;
    int n = 0, nlog = 0, f1 = 0, f2 = 0, f3 = 0;
    for (int y = height0; y <= height1; y++)
        for (int x = 0; x < w; x++) {
            float a, b;
            if (!metrics_px(gt, gw, gh, gc, given, given16, w, given_c, rx, ry, x, y, 0, cap_depth,
                            depth_max, &a, &b))
                continue;
            if (align_way == 1)
                b *= shift;
            else if (align_way == 2)
                b = b * ls_s + ls_o;
            mse = (float)((double)mse + pow(a - b, 2));
            mae += fabsf(a - b);
            mre += fabsf(a - b) / a;
            if (a > 1e-4 && b > 1e-4) {
                float lg = log10f(a) - log10f(b);
                mselog = (float)((double)mselog + pow(lg, 2));
                nlog++;
            }
            if (a > 0 && b > 0) {
                float r01 = a / b, r10 = b / a;
                float rm = r01 > r10 ? r01 : r10;
                if (rm >= 1.25) f1++;
                if (rm >= pow(1.25, 2)) f2++;
                if (rm >= pow(1.25, 3)) f3++;
            }
            n++;
        }
    out[0] = mse / (float)n;
    out[1] = mae / (float)n;
    out[2] = mre / (float)n;
    out[3] = mselog / (float)nlog;
    out[4] = (float)(n - f1) / (float)n;
    out[5] = (float)(n - f2) / (float)n;
    out[6] = (float)(n - f3) / (float)n;
    out[7] = shift;
    out[8] = ls_s;
    out[9] = ls_o;
    out[10] = gt_med;
    out[11] = gv_med;
    cnt[0] = n;
    cnt[1] = nlog;
}

/* ---------------- SolveDepthBySmoothing (Depth.cpp:1773-1878) ---------------- */
int pfo_solve_smoothing(const pfo_tile* tiles, int ntiles, const float* tile_data, int width,
                        int height, float zr0, float zr1, uint16_t* data)
{ /* Returns -1 for a degenerate box (x0 == x1: the reference never terminates), -2 when a box
   * or the smoothing stencil leaves the buffer (the reference reads/writes out of bounds).
   * Taps whose linear index leaves the tile are clamped as in pfo_targets. */
    long long n = (long long)width * height;
    float* buffer = (float*)calloc((size_t)n, sizeof(float));         /* :1775-1777 */
    unsigned char* to_smooth = (unsigned char*)calloc((size_t)n, 1);   /* :1785-1786 */
    const int range = 10;                                              /* :1787 */
    int height0 = (int)floor((double)((float)height * zr0) / MYPI);     /* :1781 */
    int height1 = (int)ceil((double)((float)height * zr1) / MYPI);      /* :1782 */
    int rc = 0;
    long long oob = 0;
    if (!buffer || !to_smooth) { rc = -3; goto done; }
    if (height0 < 1 || height1 > height - 2) { rc = -2; goto done; }
    for (int p = 0; p < ntiles; p++) { /* :1790-1835 */
        const pfo_tile* t = &tiles[p];
        int x0 = (int)round((double)t->ranges[0] / (2 * MYPI) * (double)(width - 1));
        int x1 = (int)round((double)t->ranges[1] / (2 * MYPI) * (double)(width - 1));
        int y0 = (int)round((double)t->ranges[2] / MYPI * (double)(height - 1));
        int y1 = (int)round((double)t->ranges[3] / MYPI * (double)(height - 1));
        int xs = x1 >= x0 ? 1 : -1, ys = 1;
        if (x0 == x1) { rc = -1; goto done; }
        if (x0 < 0 || x0 >= width || x1 < 0 || x1 >= width || y0 < 0 || y1 >= height) {
            rc = -2;
            goto done;
        }
        int X = x0;
        while (1) { /* X from x0 up to, but excluding, x1 */
            for (int Y = y0; Y <= y1; Y += ys) {
                float xy[2];
                pfo_sph_to_2d(t, pfo_grid_azimuth(X, width), pfo_grid_zenith(Y, height), xy);
                long long idx = clamp_index(t, pfo_tile_index(t, xy[0], xy[1]), &oob);
                buffer[(long long)Y * width + X] = tile_data[t->offset + idx];
                if (abs(X - x0) <= range || abs(X - x1) <= range || abs(Y - y0) <= range ||
                    abs(Y - y1) <= range)
                    to_smooth[(long long)Y * width + X] = 1;
            }
            X += xs;
            if (X == x1) break;
        }
    }
    for (int iter = 0; iter < 500; iter++) /* :1838-1856, in place, row-major */
        for (int Y = height0; Y <= height1; Y++)
            for (int X = 1; X < width - 1; X++) {
                long long o = (long long)Y * width + X;
                if (!to_smooth[o]) continue;
                float val = buffer[o];
                float val0 = buffer[o - 1];
                float val1 = buffer[o + 1];
                float val2 = buffer[o - width];
                float val3 = buffer[o + width];
                float avg = (val0 + val1 + val2 + val3) / 4;
                buffer[o] = (float)((double)val + 0.5 * (double)(avg - val)); /* 0.5: double */
            }
    for (long long i = 0; i < n; i++) { /* :1859-1872 */
        float val = buffer[i];
        if (val < 0) val = 0;
        if (val > 1) val = 1;
        data[i] = (uint16_t)(val * 65535.0f);
    }
done:
    free(buffer);
    free(to_smooth);
    return rc;
}
