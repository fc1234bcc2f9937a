/* Registration-gather line floor: for each tile of a layout (tiles.bin from tools/reg_floor.py),
 * the distinct 128-B lines its registration samples touch in the tile and in the baseline
 * (Depth.cpp:1328-1387, restated by oracle/pf_oracle.c pfo_reg_samples), summed.  Test/analysis
 * tooling only.  Usage: reg_lines tiles.bin ntiles ew eh zr0 zr1 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pf_oracle.h"

static int cmpll(const void* a, const void* b)
{
    long long x = *(const long long*)a, y = *(const long long*)b;
    return x < y ? -1 : x > y;
}

static long long distinct(long long* v, long long n)
{
    qsort(v, (size_t)n, sizeof(long long), cmpll);
    long long d = 0;
    for (long long i = 0; i < n; i++) d += (i == 0 || v[i] != v[i - 1]);
    return d;
}

int main(int argc, char** argv)
{
    if (argc != 7) return 2;
    const int nt = atoi(argv[2]), ew = atoi(argv[3]), eh = atoi(argv[4]);
    const float zr0 = (float)atof(argv[5]), zr1 = (float)atof(argv[6]);
    pfo_tile* t = (pfo_tile*)malloc(sizeof(pfo_tile) * nt);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(t, sizeof(pfo_tile), nt, f) != (size_t)nt) return 2;
    fclose(f);
    long long samples = 0, tile_lines = 0, emap_lines_sum = 0;
    long long* el_all = NULL;
    long long nel_all = 0;
    for (int p = 0; p < nt; p++) {
        int cols, rows;
        float zt, zd;
        pfo_reg_grid(&t[p], zr0, zr1, &cols, &rows, &zt, &zd);
        const long long n = (long long)(cols + 1) * (rows + 1);
        long long* tl = (long long*)malloc(sizeof(long long) * n);
        long long* el = (long long*)malloc(sizeof(long long) * n);
        long long k = 0;
        for (int r = 0; r <= rows; r++)
            for (int c = 0; c <= cols; c++) {
                float cx = t[p].ranges[0] + (t[p].ranges[1] - t[p].ranges[0]) * (float)c / (float)cols;
                float cy = zt + (zd - zt) * (float)r / (float)rows;
                float xy[2];
                pfo_sph_to_2d(&t[p], cx, cy, xy);
                if (xy[0] < 0) xy[0] = 0;
                if (xy[0] > 1) xy[0] = 1;
                if (xy[1] < 0) xy[1] = 0;
                if (xy[1] > 1) xy[1] = 1;
                const long long ti = t[p].offset + pfo_tile_index(&t[p], xy[0], xy[1]);
                const int x = (int)((double)cx / (PFO_MYPI * 2) * (double)(float)(ew - 1));
                const int y = (int)((double)cy / PFO_MYPI * (double)(float)(eh - 1));
                tl[k] = ti * 4 / 128;
                el[k] = ((long long)y * ew + x) * 4 / 128;
                k++;
            }
        samples += n;
        tile_lines += distinct(tl, n);
        const long long d = distinct(el, n);
        emap_lines_sum += d;
        el_all = (long long*)realloc(el_all, sizeof(long long) * (nel_all + n));
        memcpy(el_all + nel_all, el, sizeof(long long) * n);
        nel_all += n;
        free(tl);
        free(el);
    }
    const long long emap_union = distinct(el_all, nel_all);
    printf("samples %lld tile_lines %lld emap_lines_per_tile_sum %lld emap_lines_union %lld\n",
           samples, tile_lines, emap_lines_sum, emap_union);
    return 0;
}
