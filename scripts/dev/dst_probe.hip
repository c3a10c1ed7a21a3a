// Developer probe: tile_scan's disjoint sparse table (tile_common.h) against a brute-force CPU
// build for random tiles; prints mismatches.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I <csrc> scripts/dev/dst_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "tile_common.h"
using namespace bt;
__global__ void k(const int32_t* c, Agg* D) {
    __shared__ int32_t cT[64];
    __shared__ int64_t ql[128];
    __shared__ Agg Ds[6 * 64];
    const int lane = threadIdx.x;
    TileCarry cy{0, c[0]};
    tile_scan(c[lane], 64, 0, lane, cT, ql, Ds, cy);
    __syncthreads();
    for (int i = lane; i < 6 * 64; i += 64) D[i] = Ds[i];
}
static Agg one(int x) { return Agg{x, x, 0, 0}; }
static Agg mg(Agg a, Agg b) {
    Agg r; r.mx = std::max(a.mx, b.mx); r.mn = std::min(a.mn, b.mn);
    r.dd = std::max(std::max(a.dd, b.dd), a.mx - b.mn); r.du = std::max(std::max(a.du, b.du), b.mx - a.mn); return r;
}
int main() {
    int32_t h[64]; Agg got[6 * 64];
    int32_t* dc; Agg* dD; hipMalloc(&dc, sizeof h); hipMalloc(&dD, sizeof got);
    int bad = 0;
    for (int it = 0; it < 200; ++it) {
        for (int i = 0; i < 64; ++i) h[i] = 1000 + rand() % 5000;
        hipMemcpy(dc, h, sizeof h, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dc, dD);
        hipMemcpy(got, dD, sizeof got, hipMemcpyDeviceToHost);
        for (int m = 0; m < 6; ++m)
            for (int i = 0; i < 64; ++i) {
                // level m: lanes in the right half of their 2^(m+1) block hold the prefix from the
                // half's start, left-half lanes the suffix to the half's end
                const int half = 1 << m, start = i & ~(half - 1);
                Agg e;
                if (m == 0) e = one(h[i]);
                else if ((i >> m) & 1) { e = one(h[start]); for (int j = start + 1; j <= i; ++j) e = mg(e, one(h[j])); }
                else { e = one(h[i]); for (int j = i + 1; j < start + half; ++j) e = mg(e, one(h[j])); }
                const Agg g = got[(5 - m) * 64 + i];  // rows in reverse level order (dst_row)
                if (g.mx != e.mx || g.mn != e.mn || g.dd != e.dd || g.du != e.du) {
                    if (bad++ < 20) printf("it %d level %d lane %d: got (%d %d %d %d) want (%d %d %d %d)\n", it, m, i, g.mx, g.mn, g.dd, g.du, e.mx, e.mn, e.dd, e.du);
                }
            }
    }
    printf("mismatches: %d\n", bad);
    return 0;
}
