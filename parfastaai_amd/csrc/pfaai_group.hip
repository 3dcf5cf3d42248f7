// pfaai_group.hip -- the multi-device context of the C ABI (pfaai_group_*,
// include/pfaai_hip.h): SURVEY 8b's pfaai_create(ctx, device_ids, n_devices)
// with the RCCL communicator inside, the device-side counterpart of the
// reference's distributeGenomePairs (algorithm_impl.hpp:100-120).
//
// One process drives the group from one host thread: one pfaai_ctx per
// device, one RCCL communicator over the devices (ncclCommInitAll), one
// stream per device.
//   load  every device loads the caller's host arrays (one host copy feeds
//         every device, SURVEY 8e's "one pinned host buffer feeding the
//         devices"; the loads run concurrently, one host thread each) and
//         builds the walk data of its own row block only (pfaai_load_rows);
//   run   every device runs its row block (pfaai_run, asynchronous on its
//         stream) into a block buffer; the blocks are gathered into the
//         caller's device-0 arrays by grouped ncclSend / ncclRecv over xGMI
//         (ncclGather needs equal counts; the blocks are not) -- device 0
//         writes its own block in place.  PFAAI_GROUP_PEER_GATHER: no
//         communicator; each block is copied by hipMemcpyPeerAsync on
//         device 0's stream after an event of its device's run, and a device
//         may appear more than once -- so one GPU hosts an n-member group and
//         runs every piece of the n > 1 path but the RCCL calls
//         (tests/test_gpu_group.py).
// Row blocks: pfaai::split_rows with the first device's CU count (the
// row-cost model and round-tail cuts of shard.py, the cuts bench.py's ranks
// use).  ALL and QT rows map to disjoint contiguous JAC spans; QSUB rows do
// not (each row has two segments), so a QSUB problem runs on device 0 alone.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <mutex>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "pfaai_hip.h"
#include "pfaai_hip.hpp"

struct pfaai_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<pfaai_ctx*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> done;       // PEER_GATHER: a device's block is computed
    uint32_t flags = 0;
    std::vector<int64_t> cut;           // row blocks [cut[i], cut[i+1])
    std::vector<int64_t> first, count;  // their JAC spans
    std::vector<void*> blk[3];          // devices 1..n-1: block buffers of AJI, S, N
    std::vector<int64_t> blk_cap[3];    // (elements)
    int32_t mode = -1;
    bool loaded = false;
    int64_t n_rows = 0, n_pairs = 0;
    std::string err;
};

namespace {

// RCCL is opened on the first pfaai_group_create, not linked: a process that
// never makes a group (every single-device caller, and bench.py's ranks,
// whose torch.distributed carries its own librccl) loads no second copy.
// An RCCL already in the process (RTLD_NOLOAD) is reused.
struct Rccl {
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_NOLOAD)) != nullptr) break;
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if (!h && (h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!h) return;
        auto sym = [&](auto& f, const char* n) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, n)); };
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = r.CommInitAll && r.CommDestroy && r.GroupStart && r.GroupEnd && r.Send && r.Recv && r.GetErrorString;
    });
    return r;
}

int gfail(pfaai_group* g, int rc, const std::string& msg) {
    g->err = msg;
    return rc;
}

int ctx_fail(pfaai_group* g, int i, int rc) {
    return gfail(g, rc, "device " + std::to_string(g->dev[i]) + ": " + pfaai_last_error(g->ctx[i]));
}

#define GHIP(g, expr)                                                                              \
    do {                                                                                           \
        const hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return gfail(g, PFAAI_RC_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// inside an ncclGroupStart / ncclGroupEnd bracket: a failed call closes the
// bracket (a group left open defers or hangs this thread's later RCCL calls)
#define GNCCL_IN_GROUP(g, expr)                                                                    \
    do {                                                                                           \
        const ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess) {                                                                   \
            (void)rccl().GroupEnd();                                                               \
            return gfail(g, PFAAI_RC_RCCL, std::string(#expr) + ": " + rccl().GetErrorString(r_)); \
        }                                                                                          \
    } while (0)

// wait for the blocks already launched (devices < upto) before an error
// return: their kernels write the caller's or the group's buffers
void drain(pfaai_group* g, int upto) {
    for (int i = 0; i < upto && i < g->n; ++i)
        if (g->st[i]) {
            (void)hipSetDevice(g->dev[i]);
            (void)hipStreamSynchronize(g->st[i]);
        }
}

void release_blocks(pfaai_group* g) {
    for (int k = 0; k < 3; ++k) {
        for (size_t i = 0; i < g->blk[k].size(); ++i)
            if (g->blk[k][i]) {
                (void)hipSetDevice(g->dev[i]);
                (void)hipFree(g->blk[k][i]);
            }
        g->blk[k].assign(g->n, nullptr);
        g->blk_cap[k].assign(g->n, 0);
    }
}

// block buffer k (0 AJI f64, 1 S f64, 2 N i32) of device i >= 1, >= count[i] elements
int ensure_block(pfaai_group* g, int k, int i) {
    if (g->blk_cap[k][i] >= g->count[i]) return PFAAI_RC_OK;
    GHIP(g, hipSetDevice(g->dev[i]));
    if (g->blk[k][i]) GHIP(g, hipFree(g->blk[k][i]));
    g->blk[k][i] = nullptr;
    g->blk_cap[k][i] = 0;
    const size_t bytes = (size_t)g->count[i] * (k == 2 ? sizeof(int32_t) : sizeof(double));
    if (hipMalloc(&g->blk[k][i], bytes) != hipSuccess) {
        g->blk[k][i] = nullptr;
        return gfail(g, PFAAI_RC_OOM, "block buffer of " + std::to_string(bytes) + " bytes on device " +
                                          std::to_string(g->dev[i]));
    }
    g->blk_cap[k][i] = g->count[i];
    return PFAAI_RC_OK;
}

}  // namespace

extern "C" {

int pfaai_group_create_flags(pfaai_group** out, const int* device_ids, int n_devices, uint32_t flags) {
    if (!out) return PFAAI_RC_INVALID;
    *out = nullptr;
    if (!device_ids || n_devices < 1 || (flags & ~(uint32_t)PFAAI_GROUP_PEER_GATHER)) return PFAAI_RC_INVALID;
    const bool peer = flags & PFAAI_GROUP_PEER_GATHER;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return PFAAI_RC_HIP;
    for (int i = 0; i < n_devices; ++i) {
        if (device_ids[i] < 0 || device_ids[i] >= ndev) return PFAAI_RC_INVALID;
        for (int j = 0; j < i && !peer; ++j)
            if (device_ids[j] == device_ids[i]) return PFAAI_RC_INVALID;  // (one RCCL rank per device)
    }
    auto* g = new (std::nothrow) pfaai_group;
    if (!g) return PFAAI_RC_OOM;
    g->n = n_devices;
    g->flags = flags;
    g->dev.assign(device_ids, device_ids + n_devices);
    g->ctx.assign(n_devices, nullptr);
    g->st.assign(n_devices, nullptr);
    g->done.assign(n_devices, nullptr);
    g->comm.assign(n_devices, nullptr);
    release_blocks(g);
    int rc = PFAAI_RC_OK;
    for (int i = 0; i < n_devices && rc == PFAAI_RC_OK; ++i) {
        rc = pfaai_create(&g->ctx[i], g->dev[i]);
        if (rc == PFAAI_RC_OK) {
            (void)hipSetDevice(g->dev[i]);
            if (hipStreamCreateWithFlags(&g->st[i], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&g->done[i], hipEventDisableTiming) != hipSuccess)
                rc = PFAAI_RC_HIP;
        }
    }
    if (peer) {
        if (rc != PFAAI_RC_OK) {
            pfaai_group_destroy(g);
            return rc;
        }
        *out = g;
        return PFAAI_RC_OK;
    }
    if (rc == PFAAI_RC_OK && !rccl().ok) {
        g->err = "librccl.so.1 not found (or lacks a symbol)";
        rc = PFAAI_RC_RCCL;
    }
    if (rc == PFAAI_RC_OK && rccl().CommInitAll(g->comm.data(), n_devices, g->dev.data()) != ncclSuccess) {
        g->comm.assign(n_devices, nullptr);
        rc = PFAAI_RC_RCCL;
    }
    if (rc != PFAAI_RC_OK) {
        pfaai_group_destroy(g);
        return rc;
    }
    *out = g;
    return PFAAI_RC_OK;
}

int pfaai_group_create(pfaai_group** out, const int* device_ids, int n_devices) {
    return pfaai_group_create_flags(out, device_ids, n_devices, 0u);
}

int pfaai_group_destroy(pfaai_group* g) {
    if (!g) return PFAAI_RC_OK;
    for (int i = 0; i < g->n; ++i)
        if (g->st[i]) {
            (void)hipSetDevice(g->dev[i]);
            (void)hipStreamSynchronize(g->st[i]);
        }
    for (auto& c : g->comm)
        if (c) (void)rccl().CommDestroy(c);
    release_blocks(g);
    for (int i = 0; i < g->n; ++i) {
        if (g->st[i]) {
            (void)hipSetDevice(g->dev[i]);
            (void)hipStreamDestroy(g->st[i]);
        }
        if (g->done[i]) {
            (void)hipSetDevice(g->dev[i]);
            (void)hipEventDestroy(g->done[i]);
        }
        if (g->ctx[i]) pfaai_destroy(g->ctx[i]);
    }
    delete g;
    return PFAAI_RC_OK;
}

const char* pfaai_group_last_error(const pfaai_group* g) { return g ? g->err.c_str() : "null group"; }

int pfaai_group_size(const pfaai_group* g, int* n_devices) {
    if (!g || !n_devices) return PFAAI_RC_INVALID;
    *n_devices = g->n;
    return PFAAI_RC_OK;
}

pfaai_ctx* pfaai_group_ctx(pfaai_group* g, int i) { return g && i >= 0 && i < g->n ? g->ctx[i] : nullptr; }

int pfaai_group_load(pfaai_group* g, const pfaai_problem* prob) {
    if (!g || !prob) return PFAAI_RC_INVALID;
    g->loaded = false;
    const int n = g->n;
    // row blocks: ALL by the row-cost model, QT equal rows, QSUB device 0 alone
    int64_t rows = prob->mode == PFAAI_MODE_ALL ? prob->n_ids : prob->n_qry;
    if (rows < 0) return gfail(g, PFAAI_RC_INVALID, "negative row count");
    if (prob->mode == PFAAI_MODE_QSUB) {
        g->cut.assign(n + 1, rows);
        g->cut[0] = 0;
    } else {
        int cus = 0;  // the round-tail cuts of bench.py's ranks (shard.split_rows(cus=...))
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->dev[0]) != hipSuccess) cus = 0;
        g->cut = pfaai::split_rows(rows, n, prob->mode == PFAAI_MODE_ALL, cus);
    }
    // concurrent loads, one host thread per device context
    std::vector<int> rc(n, PFAAI_RC_OK);
    {
        std::vector<std::thread> th;
        for (int i = 0; i < n; ++i)
            th.emplace_back([&, i] {
                rc[i] = n > 1 && prob->mode == PFAAI_MODE_ALL
                            ? pfaai_load_rows(g->ctx[i], prob, g->cut[i], g->cut[i + 1])
                            : pfaai_load(g->ctx[i], prob);
            });
        for (auto& t : th) t.join();
    }
    for (int i = 0; i < n; ++i)
        if (rc[i] != PFAAI_RC_OK) return ctx_fail(g, i, rc[i]);
    int r;
    if ((r = pfaai_shape(g->ctx[0], &g->n_rows, &g->n_pairs))) return ctx_fail(g, 0, r);
    g->first.assign(n, 0);
    g->count.assign(n, 0);
    for (int i = 0; i < n; ++i)
        if (g->cut[i + 1] > g->cut[i] && (r = pfaai_row_span(g->ctx[0], g->cut[i], g->cut[i + 1], &g->first[i], &g->count[i])))
            return ctx_fail(g, 0, r);
    g->mode = prob->mode;
    g->loaded = true;
    return PFAAI_RC_OK;
}

int pfaai_group_blocks(const pfaai_group* g, int64_t* cuts) {
    if (!g || !cuts) return PFAAI_RC_INVALID;
    if (!g->loaded) return PFAAI_RC_INVALID;
    for (int i = 0; i <= g->n; ++i) cuts[i] = g->cut[i];
    return PFAAI_RC_OK;
}

int pfaai_group_run(pfaai_group* g, uint32_t flags, double* d_aji, double* d_S, int32_t* d_N) {
    if (!g) return PFAAI_RC_INVALID;
    if (!g->loaded) return gfail(g, PFAAI_RC_INVALID, "no problem loaded");
    if ((flags & PFAAI_FLAG_EMIT_JAC) && (!d_S || !d_N)) return gfail(g, PFAAI_RC_INVALID, "EMIT_JAC needs S and N");
    if (!d_aji && !(flags & PFAAI_FLAG_EMIT_JAC)) return gfail(g, PFAAI_RC_INVALID, "no output");
    if (flags & PFAAI_FLAG_FULL_ROWS) return gfail(g, PFAAI_RC_INVALID, "FULL_ROWS: use pfaai_stream_matrix per context");
    const bool jac = flags & PFAAI_FLAG_EMIT_JAC;
    void* out[3] = {d_aji, jac ? d_S : nullptr, jac ? d_N : nullptr};
    const size_t esz[3] = {sizeof(double), sizeof(double), sizeof(int32_t)};
    int r;
    // every device's block, asynchronously on its stream (device 0 in place)
    for (int i = 0; i < g->n; ++i) {
        if (g->cut[i + 1] <= g->cut[i]) continue;
        void* base[3] = {nullptr, nullptr, nullptr};
        for (int k = 0; k < 3; ++k) {
            if (!out[k]) continue;
            if (i == 0) {
                base[k] = out[k];
            } else {
                if ((r = ensure_block(g, k, i))) {
                    drain(g, i);
                    return r;
                }
                base[k] = static_cast<char*>(g->blk[k][i]) - (ptrdiff_t)(g->first[i] * (int64_t)esz[k]);
            }
        }
        if ((r = pfaai_run(g->ctx[i], g->cut[i], g->cut[i + 1], flags, static_cast<double*>(base[0]),
                           static_cast<double*>(base[1]), static_cast<int32_t*>(base[2]), g->st[i]))) {
            drain(g, g->n);
            return ctx_fail(g, i, r);
        }
    }
    if (g->n > 1 && (g->flags & PFAAI_GROUP_PEER_GATHER)) {
        // the gather by peer copies on device 0's stream, each after its block
        for (int i = 1; i < g->n; ++i) {
            if (g->count[i] <= 0) continue;
            GHIP(g, hipSetDevice(g->dev[i]));
            GHIP(g, hipEventRecord(g->done[i], g->st[i]));
            GHIP(g, hipSetDevice(g->dev[0]));
            GHIP(g, hipStreamWaitEvent(g->st[0], g->done[i], 0));
            for (int k = 0; k < 3; ++k) {
                if (!out[k]) continue;
                GHIP(g, hipMemcpyPeerAsync(static_cast<char*>(out[k]) + g->first[i] * (int64_t)esz[k], g->dev[0],
                                           g->blk[k][i], g->dev[i], (size_t)g->count[i] * esz[k], g->st[0]));
            }
        }
    } else if (g->n > 1) {
        // the gather into device 0's arrays: grouped point-to-point transfers
        const Rccl& R = rccl();
        if (R.GroupStart() != ncclSuccess) {
            drain(g, g->n);
            return gfail(g, PFAAI_RC_RCCL, "ncclGroupStart failed");
        }
        for (int i = 1; i < g->n; ++i) {
            if (g->count[i] <= 0) continue;
            for (int k = 0; k < 3; ++k) {
                if (!out[k]) continue;
                const ncclDataType_t t = k == 2 ? ncclInt32 : ncclFloat64;
                GNCCL_IN_GROUP(g, R.Send(g->blk[k][i], (size_t)g->count[i], t, 0, g->comm[i], g->st[i]));
                GNCCL_IN_GROUP(g, R.Recv(static_cast<char*>(out[k]) + g->first[i] * (int64_t)esz[k], (size_t)g->count[i], t,
                                         i, g->comm[0], g->st[0]));
            }
        }
        const ncclResult_t re = R.GroupEnd();
        if (re != ncclSuccess) {
            drain(g, g->n);
            return gfail(g, PFAAI_RC_RCCL, std::string("ncclGroupEnd: ") + R.GetErrorString(re));
        }
    }
    for (int i = 0; i < g->n; ++i) {
        GHIP(g, hipSetDevice(g->dev[i]));
        GHIP(g, hipStreamSynchronize(g->st[i]));
    }
    return PFAAI_RC_OK;
}

}  // extern "C"
