// comm.cpp — the multi-GPU exchange step behind the C ABI: one RCCL
// all-gather over xGMI of every rank's top-k records and run counters, straight from the
// engine's device buffers, then the host merge with the engine's order.
//
// The reference's only parallelism is file-level job farming over gRPC
// (/root/reference/src/server/main.rs:131-143) with no collective at all. Here each GPU runs a
// contiguous block of symbols with no data-path collective; once per run the ranks exchange
// [header record | k records | bar-evals | trades] (k = 100: 2.4 KB per rank). That message is
// latency-bound, so it is a single ncclAllGather on the engine's top-k stream, enqueued behind
// the run's top-k chain without a host wait, and read back into one of BT_PIPE_SLOTS pinned slots so the
// next run overlaps it (the same pipelining as bt_topk_fetch_async / bt_topk_fetch_wait).
//
// RCCL is resolved with dlopen on the first communicator call, not linked: a single-GPU worker
// (configs 1-2) loads libbt.so on a box without librccl (the reference's worker build hook,
// /root/reference/build.rs:1-4, links nothing either). rccl.h is used for its types only. In a
// process that already holds an RCCL (PyTorch-ROCm's bundled librccl.so, SONAME librccl.so.1),
// dlopen by SONAME returns that copy, as the dynamic linker did when libbt.so linked it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "internal.h"

using namespace bt;

struct bt_comm {
    ncclComm_t comm = nullptr;
    int32_t rank = 0, world = 1, device = 0, k = 0;
    size_t rec_bytes = 0;              // bytes one rank contributes
    unsigned char* d_send = nullptr;   // [rec_bytes]
    unsigned char* d_recv[BT_PIPE_SLOTS] = {};  // [world * rec_bytes] per slot
    unsigned char* h_recv[BT_PIPE_SLOTS] = {};  // pinned
    int64_t* h_evals[BT_PIPE_SLOTS] = {};       // pinned: this rank's bar-evals per slot
    hipEvent_t done[BT_PIPE_SLOTS] = {};
    bool armed[BT_PIPE_SLOTS] = {};
};

namespace {

struct CommFail {
    std::string msg;
};

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) throw CommFail{std::string(#x) + ": " + hipGetErrorString(e_)}; \
    } while (0)

// the RCCL entry points this file calls
struct Rccl {
    void* so = nullptr;
    std::string why;  // dlopen / dlsym failure
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.so) break;
        }
        if (!r.so) {
            const char* e = dlerror();
            r.why = std::string("RCCL is not loadable (librccl.so.1): ") + (e ? e : "dlopen failed");
            return;
        }
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(r.so, name));
            if (!fn && r.why.empty()) r.why = std::string("RCCL lacks ") + name;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.AllGather, "ncclAllGather");
        sym(r.GetErrorString, "ncclGetErrorString");
    });
    if (!r.why.empty()) throw CommFail{r.why};
    return r;
}

#define NCCLCHK(x)                                                                             \
    do {                                                                                       \
        ncclResult_t r_ = (x);                                                                 \
        if (r_ != ncclSuccess)                                                                 \
            throw CommFail{std::string(#x) + ": " + rccl().GetErrorString(r_)};               \
    } while (0)

// Per-rank message: header record (record count in its first int32), k records, then the two
// int64 counters (bar-evals, trades).
size_t message_bytes(int32_t k) { return ((size_t)k + 1) * sizeof(bt_topk_rec) + 2 * sizeof(int64_t); }

// The host half of bt_exchange_wait: merge `world` gathered messages of k_msg records each.
int32_t merge_block(const unsigned char* block, int32_t world, int32_t k_msg, bt_topk_rec* out,
                    int32_t k, int64_t* counters) {
    const size_t mb = message_bytes(k_msg);
    std::vector<bt_topk_rec> all;
    all.reserve((size_t)k_msg * world);
    int64_t evals = 0, trades = 0;
    for (int32_t r = 0; r < world; ++r) {
        const unsigned char* m = block + (size_t)r * mb;
        int32_t n = 0;
        memcpy(&n, m, sizeof n);
        // every rank's device selection is exact whatever the ties (k_topk.hip
        // topk_finish_ties), so a tie-heavy grid exchanges like any other
        if (n < 0) throw CommFail{"rank " + std::to_string(r) + ": bad top-k record count"};
        n = std::min(n, k_msg);
        const unsigned char* recs = m + sizeof(bt_topk_rec);
        for (int32_t i = 0; i < n; ++i) {  // memcpy: the block carries no alignment promise
            bt_topk_rec x;
            memcpy(&x, recs + (size_t)i * sizeof x, sizeof x);
            all.push_back(x);
        }
        int64_t x[2];
        memcpy(x, m + ((size_t)k_msg + 1) * sizeof(bt_topk_rec), sizeof x);
        evals += x[0];
        trades += x[1];
    }
    const size_t mm = std::min<size_t>(all.size(), (size_t)std::min(k, k_msg));
    std::partial_sort(all.begin(), all.begin() + mm, all.end(), topk_less);
    std::copy(all.begin(), all.begin() + mm, out);
    if (counters) {
        counters[0] = evals;
        counters[1] = trades;
    }
    return (int32_t)mm;
}

void release(bt_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (int s = 0; s < BT_PIPE_SLOTS; ++s) {
        if (c->done[s]) (void)hipEventSynchronize(c->done[s]);
    }
    if (c->comm) (void)rccl().CommDestroy(c->comm);  // comm set: rccl() resolved
    if (c->d_send) (void)hipFree(c->d_send);
    for (int s = 0; s < BT_PIPE_SLOTS; ++s) {
        if (c->d_recv[s]) (void)hipFree(c->d_recv[s]);
        if (c->h_recv[s]) (void)hipHostFree(c->h_recv[s]);
        if (c->h_evals[s]) (void)hipHostFree(c->h_evals[s]);
        if (c->done[s]) (void)hipEventDestroy(c->done[s]);
    }
    delete c;
}

}  // namespace

extern "C" {

int32_t bt_comm_unique_id(uint8_t* out) {
    try {
        if (!out) throw CommFail{"null output"};
        ncclUniqueId id;
        NCCLCHK(rccl().GetUniqueId(&id));
        static_assert(sizeof(id) == BT_COMM_ID_BYTES, "RCCL unique id size");
        memcpy(out, &id, sizeof id);
        return 0;
    } catch (const CommFail& f) {
        set_last_error(f.msg);
        return -1;
    } catch (...) {
        set_last_error("unknown exception");
        return -1;
    }
}

bt_comm* bt_comm_create(const uint8_t* id, int32_t rank, int32_t world, int32_t device,
                        int32_t k, char* err, size_t errlen) {
    bt_comm* c = nullptr;
    try {
        if (!id || world < 1 || rank < 0 || rank >= world || k < 1 || k > 1024)
            throw CommFail{"bad arguments"};
        c = new bt_comm();
        c->rank = rank;
        c->world = world;
        c->device = device;
        c->k = k;
        c->rec_bytes = message_bytes(k);
        const Rccl& nc = rccl();
        HIPCHK(hipSetDevice(device));
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof uid);
        NCCLCHK(nc.CommInitRank(&c->comm, world, uid, rank));
        HIPCHK(hipMalloc(&c->d_send, c->rec_bytes));
        for (int s = 0; s < BT_PIPE_SLOTS; ++s) {
            HIPCHK(hipMalloc(&c->d_recv[s], c->rec_bytes * world));
            HIPCHK(hipHostMalloc(&c->h_recv[s], c->rec_bytes * world));
            HIPCHK(hipHostMalloc(&c->h_evals[s], sizeof(int64_t)));
            HIPCHK(hipEventCreateWithFlags(&c->done[s], hipEventDisableTiming));
        }
        return c;
    } catch (const CommFail& f) {
        release(c);
        set_last_error(f.msg);
        if (err && errlen) snprintf(err, errlen, "%s", f.msg.c_str());
        return nullptr;
    } catch (...) {
        release(c);
        set_last_error("unknown exception");
        if (err && errlen) snprintf(err, errlen, "unknown exception");
        return nullptr;
    }
}

void bt_comm_destroy(bt_comm* c) { release(c); }

int32_t bt_exchange_async(bt_comm* c, bt_engine* e, int32_t slot) {
    try {
        if (!c || !e || slot < 0 || slot >= BT_PIPE_SLOTS) throw CommFail{"bad arguments"};
        ExchangeView v{};
        std::string why;
        if (!engine_exchange_view(e, v, why)) throw CommFail{why};
        if (v.device != c->device) throw CommFail{"engine and communicator are on different devices"};
        if (v.topk < c->k) throw CommFail{"engine topk is smaller than the communicator's k"};
        HIPCHK(hipSetDevice(c->device));
        // the slot's previous read-back must be consumed before its pinned buffers are reused
        if (c->armed[slot]) HIPCHK(hipEventSynchronize(c->done[slot]));
        const size_t recs = ((size_t)c->k + 1) * sizeof(bt_topk_rec);
        unsigned char* cnt = c->d_send + recs;
        *c->h_evals[slot] = v.bar_evals;
        // header + the first k records of the run's top-k, its trade counter, its bar-evals
        HIPCHK(hipMemcpyAsync(c->d_send, v.d_top, recs, hipMemcpyDeviceToDevice, v.tstream));
        HIPCHK(hipMemcpyAsync(cnt, c->h_evals[slot], sizeof(int64_t), hipMemcpyHostToDevice, v.tstream));
        HIPCHK(hipMemcpyAsync(cnt + sizeof(int64_t), v.d_ntr, sizeof(int64_t), hipMemcpyDeviceToDevice,
                              v.tstream));
        engine_exchange_enqueued(e);
        NCCLCHK(rccl().AllGather(c->d_send, c->d_recv[slot], c->rec_bytes, ncclChar, c->comm,
                                 v.tstream));
        HIPCHK(hipMemcpyAsync(c->h_recv[slot], c->d_recv[slot], c->rec_bytes * c->world,
                              hipMemcpyDeviceToHost, v.tstream));
        HIPCHK(hipEventRecord(c->done[slot], v.tstream));
        c->armed[slot] = true;
        return 0;
    } catch (const CommFail& f) {
        set_last_error(f.msg);
        return -1;
    } catch (...) {
        set_last_error("unknown exception");
        return -1;
    }
}

int32_t bt_exchange_wait(bt_comm* c, int32_t slot, bt_topk_rec* out, int32_t k,
                         int64_t* counters) {
    try {
        if (!c || slot < 0 || slot >= BT_PIPE_SLOTS || !out || k < 1) throw CommFail{"bad arguments"};
        if (!c->armed[slot]) throw CommFail{"no exchange pending on this slot"};
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipEventSynchronize(c->done[slot]));
        c->armed[slot] = false;
        return merge_block(c->h_recv[slot], c->world, c->k, out, k, counters);
    } catch (const CommFail& f) {
        set_last_error(f.msg);
        return -1;
    } catch (...) {
        set_last_error("unknown exception");
        return -1;
    }
}

int64_t bt_exchange_message_bytes(int32_t k) { return k < 1 ? -1 : (int64_t)message_bytes(k); }

int32_t bt_exchange_merge(const uint8_t* block, size_t block_bytes, int32_t world, int32_t k_msg,
                          bt_topk_rec* out, int32_t k, int64_t* counters) {
    try {
        if (!block || world < 1 || k_msg < 1 || !out || k < 1) throw CommFail{"bad arguments"};
        // a short or mismatched block (a truncated gather, a rank that sent another k) is
        // rejected, never read past its end
        if (block_bytes != (size_t)world * message_bytes(k_msg))
            throw CommFail{"block holds " + std::to_string(block_bytes) + " bytes, not world x " +
                           std::to_string(message_bytes(k_msg))};
        return merge_block(block, world, k_msg, out, k, counters);
    } catch (const CommFail& f) {
        set_last_error(f.msg);
        return -1;
    } catch (...) {
        set_last_error("unknown exception");
        return -1;
    }
}

}  // extern "C"
