// k_lane.hip — EMA+rolling-OLS (config 3) and Bollinger+SL/TP (config 4) backtests:
// one lane per (symbol, parameter), the path-dependent state machine walked bar by bar.
//
// Spec: docs/oracle_spec.md §3-§5; checked bit-for-bit against oracle/oracle.c
// (orc_ema_ols, orc_boll). Replaces the sleep in process_incoming_job
// (/root/reference/src/worker/process.rs:21-25) for these strategies.
//
// Per-bar symbol data (close, high, low, q, q2) is the same address for every lane of a
// workgroup (one symbol per workgroup row), so it is a broadcast load; each lane keeps its
// EMA, OLS window sums / Bollinger window sums and its trade accounting in registers.
#include "device_common.h"

namespace bt {

// Fixed-point returns per (symbol, bar): q[off+t], q2[off+t] (spec §3); q[off] = 0.
__global__ __launch_bounds__(256) void ret_kernel(const SymDesc* __restrict__ syms,
                                                  const int32_t* __restrict__ close,
                                                  int64_t* __restrict__ q, int64_t* __restrict__ q2) {
    const SymDesc sd = syms[blockIdx.y];
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < sd.bars; t += gridDim.x * blockDim.x) {
        int64_t a = 0, b = 0;
        if (t >= 1) fixed_ret(close[sd.off + t], close[sd.off + t - 1], a, b);
        q[sd.off + t] = a;
        q2[sd.off + t] = b;
    }
}

struct BarAcct {
    int32_t pos, e, ntr;
    int64_t ce, R, peak, mdd, expo;
    i128 s1, s2;
    uint64_t h;
};

__device__ __forceinline__ void bar_init(BarAcct& a) {
    a.pos = a.e = a.ntr = 0;
    a.ce = a.R = a.peak = a.mdd = a.expo = 0;
    a.s1 = a.s2 = 0;
    a.h = kFnvOff;
}

__device__ __forceinline__ void bar_returns(BarAcct& a, int64_t q, int64_t q2) {
    if (a.pos == 0) return;
    a.s1 += (i128)(a.pos > 0 ? q : -q);
    a.s2 += (i128)q2;
    a.expo += 1;
}

__device__ __forceinline__ void bar_close(BarAcct& a, int t, int64_t px, bt_trade* tr, int cap) {
    a.R += a.pos > 0 ? px - a.ce : a.ce - px;
    const uint64_t w = (uint64_t)(uint32_t)a.e | ((uint64_t)(uint32_t)t << 31) |
                       ((uint64_t)(a.pos > 0) << 62);
    a.h = (a.h ^ w) * kFnvPrime;
    if (tr != nullptr && a.ntr < cap) {
        bt_trade r;
        r.entry_bar = a.e;
        r.exit_bar = t;
        r.side = a.pos;
        r.pad = 0;
        r.entry_px = a.ce;
        r.exit_px = px;
        tr[a.ntr] = r;
    }
    a.ntr++;
    a.pos = 0;
}

__device__ __forceinline__ void bar_equity(BarAcct& a, int64_t c) {
    const int64_t E = a.pos == 0 ? a.R : (a.pos > 0 ? a.R + (c - a.ce) : a.R + (a.ce - c));
    a.peak = max(a.peak, E);
    a.mdd = max(a.mdd, a.peak - E);
}

__device__ __forceinline__ void bar_write(const BarAcct& a, int bars, double sqrt_ann, size_t gi,
                                          const Out& out) {
    const uint64_t s1lo = (uint64_t)a.s1, s2lo = (uint64_t)a.s2;
    const int64_t s1hi = (int64_t)(a.s1 >> 64), s2hi = (int64_t)(a.s2 >> 64);
    const double sh = sharpe_fx(s1lo, s1hi, s2lo, s2hi, bars, sqrt_ann);
    bt_summary r;
    r.n_trades = a.ntr;
    r.status = 0;
    r.pnl = a.R;
    r.mdd = a.mdd;
    r.exposure = a.expo;
    r.sharpe = sh;
    r.hash = a.h;
    out.sum[gi] = r;
    out.key[gi] = order_key(sh);
    if (out.sums != nullptr) out.sums[gi] = bt_sums{s1lo, s1hi, s2lo, s2hi};
}

template <bool PARITY>
__global__ __launch_bounds__(256) void ema_ols_kernel(const SymDesc* __restrict__ syms,
                                                      const int32_t* __restrict__ close,
                                                      const int64_t* __restrict__ q,
                                                      const int64_t* __restrict__ q2, Grid g,
                                                      Out out) {
    const SymDesc sd = syms[blockIdx.x];
    const int P = g.n_params;
    const int p = blockIdx.y * blockDim.x + threadIdx.x;
    const bool active = p < P;
    const int pp = active ? p : 0;
    const int n = g.a[pp / g.nb], w = g.b[pp % g.nb];
    const int B = sd.bars;
    const int32_t* c = close + sd.off;
    const int64_t* qq = q + sd.off;
    const int64_t* qq2 = q2 + sd.off;
    const double alpha = 2.0 / ((double)n + 1.0);
    const double lo_mult = (double)(10000 - g.band_bps), hi_mult = (double)(10000 + g.band_bps);
    const int warm = (n > w ? n : w) - 1;
    const size_t gi = (size_t)blockIdx.x * P + p;
    bt_trade* tr = (PARITY && active) ? out.trades + gi * out.trade_cap : nullptr;
    BarAcct a;
    bar_init(a);
    double e = 0.0;
    int64_t S = 0, T = 0;
    if (active) {
        for (int t = 0; t < B; ++t) {
            const int32_t ct = c[t];
            e = t == 0 ? (double)ct : e + alpha * ((double)ct - e);
            if (t < w) {
                S += ct;
                T += (int64_t)t * ct;
            } else {
                const int64_t old = c[t - w];
                T = T - (S - old) + (int64_t)(w - 1) * ct;
                S = S - old + ct;
            }
            bar_returns(a, qq[t], qq2[t]);
            int np = a.pos;
            if (t == B - 1) {
                np = 0;
            } else if (t >= warm) {
                const int64_t N = 2 * T - (int64_t)(w - 1) * S;
                const double cd = (double)ct;
                if (a.pos == 1) {
                    if (cd >= e) np = 0;
                } else if (a.pos == -1) {
                    if (cd <= e) np = 0;
                } else {
                    const double lhs = cd * 10000.0;
                    const double lo = e * lo_mult, hi = e * hi_mult;
                    if (lhs < lo && N >= 0) np = 1;
                    else if (lhs > hi && N <= 0) np = -1;
                }
            }
            if (np != a.pos) {
                if (a.pos != 0) bar_close(a, t, ct, tr, out.trade_cap);
                if (np != 0) {
                    a.pos = np;
                    a.e = t;
                    a.ce = ct;
                }
            }
            bar_equity(a, ct);
        }
        bar_write(a, B, g.sqrt_ann, gi, out);
    }
    wave_add_trades(out, active ? a.ntr : 0);
}

template <bool PARITY>
__global__ __launch_bounds__(256) void boll_kernel(const SymDesc* __restrict__ syms,
                                                   const int32_t* __restrict__ high,
                                                   const int32_t* __restrict__ low,
                                                   const int32_t* __restrict__ close,
                                                   const int64_t* __restrict__ q,
                                                   const int64_t* __restrict__ q2, Grid g,
                                                   Out out) {
    const SymDesc sd = syms[blockIdx.x];
    const int P = g.n_params;
    const int p = blockIdx.y * blockDim.x + threadIdx.x;
    const bool active = p < P;
    const int pp = active ? p : 0;
    // param = ((iw * nk + ik) * nsl + isl) * ntp + itp
    const int itp = pp % g.nd, isl = (pp / g.nd) % g.nc, ik = (pp / (g.nd * g.nc)) % g.nb,
              iw = pp / (g.nd * g.nc * g.nb);
    const int w = g.a[iw];
    const int64_t kn = g.b[ik], kd = g.k_den;
    const int64_t sl = g.c[isl], tp = g.d[itp];
    const i128 kd2 = (i128)(kd * kd), kn2 = (i128)(kn * kn);
    const int B = sd.bars;
    const int32_t* c = close + sd.off;
    const int32_t* hh = high + sd.off;
    const int32_t* ll = low + sd.off;
    const int64_t* qq = q + sd.off;
    const int64_t* qq2 = q2 + sd.off;
    const size_t gi = (size_t)blockIdx.x * P + p;
    bt_trade* tr = (PARITY && active) ? out.trades + gi * out.trade_cap : nullptr;
    BarAcct a;
    bar_init(a);
    int64_t Sc = 0, sl_l = 0, tp_l = 0;
    i128 Sc2 = 0;
    if (active) {
        for (int t = 0; t < B; ++t) {
            const int64_t ct = c[t];
            Sc += ct;
            Sc2 += (i128)(ct * ct);
            if (t >= w) {
                const int64_t old = c[t - w];
                Sc -= old;
                Sc2 -= (i128)(old * old);
            }
            bar_returns(a, qq[t], qq2[t]);
            bool exited = false;
            if (a.pos != 0 && t >= a.e + 1) {
                const int64_t ht = hh[t], lt = ll[t];
                if (a.pos == 1) {
                    if (lt <= sl_l) { bar_close(a, t, sl_l, tr, out.trade_cap); exited = true; }
                    else if (ht >= tp_l) { bar_close(a, t, tp_l, tr, out.trade_cap); exited = true; }
                } else {
                    if (ht >= sl_l) { bar_close(a, t, sl_l, tr, out.trade_cap); exited = true; }
                    else if (lt <= tp_l) { bar_close(a, t, tp_l, tr, out.trade_cap); exited = true; }
                }
            }
            if (t == B - 1) {
                if (a.pos != 0) bar_close(a, t, ct, tr, out.trade_cap);
            } else if (t >= w - 1) {
                const int64_t D = (int64_t)w * ct - Sc;
                if (a.pos == 1 && D >= 0) {
                    bar_close(a, t, ct, tr, out.trade_cap);
                } else if (a.pos == -1 && D <= 0) {
                    bar_close(a, t, ct, tr, out.trade_cap);
                } else if (a.pos == 0 && !exited) {
                    const i128 Q = (i128)w * Sc2 - (i128)Sc * (i128)Sc;
                    const i128 lhs = (i128)D * (i128)D * kd2;
                    const i128 rhs = kn2 * Q;
                    if (D < 0 && lhs > rhs) {
                        a.pos = 1;
                        a.e = t;
                        a.ce = ct;
                        sl_l = ct * (10000 - sl) / 10000;
                        tp_l = ct * (10000 + tp) / 10000;
                    } else if (D > 0 && lhs > rhs) {
                        a.pos = -1;
                        a.e = t;
                        a.ce = ct;
                        sl_l = ct * (10000 + sl) / 10000;
                        tp_l = ct * (10000 - tp) / 10000;
                    }
                }
            }
            bar_equity(a, ct);
        }
        bar_write(a, B, g.sqrt_ann, gi, out);
    }
    wave_add_trades(out, active ? a.ntr : 0);
}

static hipError_t launch_ret(const SymDesc* syms, int32_t n_sym, const int32_t* close, int64_t* q,
                             int64_t* q2, hipStream_t st) {
    hipLaunchKernelGGL(ret_kernel, dim3(16, n_sym), dim3(256), 0, st, syms, close, q, q2);
    return hipGetLastError();
}

hipError_t launch_ema_ols(const SymDesc* syms, int32_t n_sym, const int32_t* close,
                          int64_t* g_q, int64_t* g_q2, const Grid& g, const Out& out, bool parity,
                          hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    hipError_t err = launch_ret(syms, n_sym, close, g_q, g_q2, st);
    if (err != hipSuccess) return err;
    const int P = g.n_params;
    const int block = P >= 256 ? 256 : ((P + 63) / 64) * 64;
    const dim3 grid(n_sym, (P + block - 1) / block);
    if (parity)
        hipLaunchKernelGGL(ema_ols_kernel<true>, grid, dim3(block), 0, st, syms, close, g_q, g_q2, g, out);
    else
        hipLaunchKernelGGL(ema_ols_kernel<false>, grid, dim3(block), 0, st, syms, close, g_q, g_q2, g, out);
    return hipGetLastError();
}

hipError_t launch_boll(const SymDesc* syms, int32_t n_sym, const int32_t* high,
                       const int32_t* low, const int32_t* close, int64_t* g_q, int64_t* g_q2,
                       const Grid& g, const Out& out, bool parity, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    hipError_t err = launch_ret(syms, n_sym, close, g_q, g_q2, st);
    if (err != hipSuccess) return err;
    const int P = g.n_params;
    const int block = P >= 256 ? 256 : ((P + 63) / 64) * 64;
    const dim3 grid(n_sym, (P + block - 1) / block);
    if (parity)
        hipLaunchKernelGGL(boll_kernel<true>, grid, dim3(block), 0, st, syms, high, low, close, g_q, g_q2, g, out);
    else
        hipLaunchKernelGGL(boll_kernel<false>, grid, dim3(block), 0, st, syms, high, low, close, g_q, g_q2, g, out);
    return hipGetLastError();
}

}  // namespace bt
