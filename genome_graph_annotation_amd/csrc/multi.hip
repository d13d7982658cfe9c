// multi.hip -- one process, N GPUs: a replica of the tree per device and
// get_rows over a batch cut into N contiguous slices, reassembled into the
// caller's ONE CSR (include/mbrwt.h "multi-device").  The reference's
// `annograph classify` is one process with a ThreadPool (main.cpp:462-497);
// this lets its C++ host drive every GPU of the node through the C ABI.
//
// Reassembly: the replicas' slice CSRs go straight to their places in the
// caller's output -- host buffers by device-to-host copies at the slice's
// label offset, device buffers (on the first device) by peer copies over
// xGMI -- after one exchange of the slice label counts on the host.  A
// gather into one buffer is exactly a set of peer copies (no collective:
// RCCL has no gatherv and the sizes are host integers already).
#include <algorithm>
#include <cstring>
#include <exception>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {
namespace {

__global__ __launch_bounds__(256) void k_rebase(uint64_t *off, uint64_t n, uint64_t add) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) gst(off + i, gld(off + i) + add);
}

}  // namespace
}  // namespace mbrwt

using namespace mbrwt;

struct mbrwt_multi {
    std::vector<mbrwt_ctx *> ctx;
    std::vector<int> dev;
    std::vector<hipStream_t> stream;
    std::vector<Workspace> rows, off, cols;  // per replica, on its device
    std::mutex mu;
};

namespace {

void slice(uint64_t n, uint32_t k, uint32_t r, uint64_t &lo, uint64_t &hi) {
    const uint64_t base = n / k, extra = n % k;
    lo = r * base + std::min<uint64_t>(r, extra);
    hi = lo + base + (r < extra ? 1 : 0);
}

void destroy(mbrwt_multi *m) {
    if (!m) return;
    for (size_t r = 0; r < m->ctx.size(); ++r) {
        if (hipSetDevice(m->dev[r]) != hipSuccess) {  // no such device: nothing was created there
            (void)hipGetLastError();                   // (and no sticky error left for the caller)
            continue;
        }
        for (Workspace *w : {&m->rows[r], &m->off[r], &m->cols[r]})
            if (w->buf) (void)hipFree(w->buf);
        if (m->stream[r]) (void)hipStreamDestroy(m->stream[r]);
        mbrwt_destroy(m->ctx[r]);
    }
    delete m;
}

// one replica per device entry, built concurrently (one host thread each)
template <class Create>
int create_multi(const int *devices, int n, mbrwt_multi **out, Create &&create) {
    if (!out || !devices || n < 1) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    mbrwt_multi *m = new (std::nothrow) mbrwt_multi();
    if (!m) return MBRWT_ERR_NOMEM;
    m->dev.assign(devices, devices + n);
    m->ctx.assign(n, nullptr);
    m->stream.assign(n, nullptr);
    m->rows.resize(n);
    m->off.resize(n);
    m->cols.resize(n);
    std::vector<int> rc(n, MBRWT_OK);
    std::vector<std::string> err(n);
    {
        std::vector<std::thread> pool;
        try {
            for (int r = 0; r < n; ++r)
                pool.emplace_back([&, r]() {
                    rc[r] = create(m->dev[r], &m->ctx[r]);
                    if (rc[r]) err[r] = mbrwt_last_error_message();
                    else if (hipSetDevice(m->dev[r]) != hipSuccess ||
                             hipStreamCreateWithFlags(&m->stream[r], hipStreamNonBlocking) != hipSuccess)
                        rc[r] = MBRWT_ERR_DEVICE;
                });
        } catch (...) {
            for (auto &t : pool) t.join();
            destroy(m);
            return MBRWT_ERR_NOMEM;
        }
        for (auto &t : pool) t.join();
    }
    for (int r = 0; r < n; ++r)
        if (rc[r]) {
            set_error("replica on device " + std::to_string(m->dev[r]) + ": " + err[r]);
            const int s = rc[r];
            destroy(m);
            return s;
        }
    *out = m;
    return MBRWT_OK;
}

// the slices on every replica: slice r's CSR in replica r's workspaces, its
// label count in need[r]; MBRWT_ERR_CAPACITY never reaches the caller here
// (the workspaces grow to the slice's size)
int run_slices(mbrwt_multi &m, const uint64_t *rows, bool rows_on_host, uint64_t n, std::vector<uint64_t> &need,
               hipStream_t s0) {
    const uint32_t k = (uint32_t)m.ctx.size();
    need.assign(k, 0);
    std::vector<int> rc(k, MBRWT_OK);
    std::vector<std::string> err(k);
    hipEvent_t ready = nullptr;
    if (!rows_on_host) {  // the caller's rows are on device 0, ordered on its stream
        if (hipSetDevice(m.dev[0]) != hipSuccess || hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(ready, s0) != hipSuccess)
            return hip_fail(hipGetLastError(), "multi: rows event");
    }
    auto one = [&](uint32_t r) -> int {
        uint64_t lo, hi;
        slice(n, k, r, lo, hi);
        const uint64_t nr = hi - lo;
        MBRWT_HIP(hipSetDevice(m.dev[r]));
        int st;
        if ((st = ensure(m.rows[r], std::max<uint64_t>(nr, 1) * 8))) return st;
        if ((st = ensure(m.off[r], (nr + 1) * 8))) return st;
        if ((st = ensure(m.cols[r], 1024 * 4))) return st;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(m.rows[r].buf);
        if (nr) {
            if (rows_on_host) {
                MBRWT_HIP(hipMemcpyAsync(d_rows, rows + lo, nr * 8, hipMemcpyHostToDevice, m.stream[r]));
            } else {
                MBRWT_HIP(hipStreamWaitEvent(m.stream[r], ready, 0));
                MBRWT_HIP(hipMemcpyPeerAsync(d_rows, m.dev[r], rows + lo, m.dev[0], nr * 8, m.stream[r]));
            }
        }
        uint64_t nd = 0;
        st = mbrwt_get_rows_device(m.ctx[r], d_rows, nr, reinterpret_cast<uint64_t *>(m.off[r].buf),
                                   reinterpret_cast<uint32_t *>(m.cols[r].buf), m.cols[r].bytes / 4, &nd, m.stream[r]);
        if (st == MBRWT_ERR_CAPACITY) {  // grow to the slice's size and run again
            if ((st = ensure(m.cols[r], (nd + nd / 8 + 1024) * 4))) return st;
            st = mbrwt_get_rows_device(m.ctx[r], d_rows, nr, reinterpret_cast<uint64_t *>(m.off[r].buf),
                                       reinterpret_cast<uint32_t *>(m.cols[r].buf), m.cols[r].bytes / 4, &nd,
                                       m.stream[r]);
        }
        need[r] = nd;
        return st;
    };
    std::vector<std::thread> pool;
    try {
        for (uint32_t r = 1; r < k; ++r)
            pool.emplace_back([&, r]() {
                rc[r] = one(r);
                if (rc[r]) err[r] = mbrwt_last_error_message();
            });
    } catch (...) {
        for (auto &t : pool) t.join();
        if (ready) (void)hipEventDestroy(ready);
        return MBRWT_ERR_NOMEM;
    }
    rc[0] = one(0);
    if (rc[0]) err[0] = mbrwt_last_error_message();
    for (auto &t : pool) t.join();
    if (ready) {
        (void)hipSetDevice(m.dev[0]);
        (void)hipEventDestroy(ready);
    }
    for (uint32_t r = 0; r < k; ++r)
        if (rc[r]) {
            set_error(err[r]);
            return rc[r];
        }
    return MBRWT_OK;
}

// the caller thread's build options (include/mbrwt.h mbrwt_set_build_option:
// thread-local), captured once and applied in every replica's worker thread
struct BuildOptions {
    int layout = build_layout(), footprint = rows_footprint(), partitioner = build_partitioner();
    BuildTuning tuning = build_tuning();
    void apply() const {
        set_build_layout(layout);
        set_rows_footprint(footprint);
        set_build_partitioner(partitioner);
        set_build_tuning(tuning);
    }
};

}  // namespace

extern "C" {

int mbrwt_multi_create(const mbrwt_tree_desc *desc, const int *devices, int n, mbrwt_multi **out) {
    if (!desc) {
        set_error("null tree description");
        return MBRWT_ERR_INVALID;
    }
    const BuildOptions opt;  // the caller thread's options, for every replica
    return create_multi(devices, n, out, [&](int d, mbrwt_ctx **c) {
        opt.apply();
        return mbrwt_create(desc, d, c);
    });
}

int mbrwt_multi_create_synthetic(const mbrwt_synth_desc *desc, const int *devices, int n, mbrwt_multi **out) {
    if (!desc) {
        set_error("null synthetic description");
        return MBRWT_ERR_INVALID;
    }
    const BuildOptions opt;
    return create_multi(devices, n, out, [&](int d, mbrwt_ctx **c) {
        opt.apply();
        return mbrwt_create_synthetic(desc, d, c);
    });
}

int mbrwt_multi_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, const int *devices, int n,
                     mbrwt_multi **out) {
    if (!bytes && len) {
        set_error("null stream");
        return MBRWT_ERR_INVALID;
    }
    mbrwt_tree *t = nullptr;  // parsed once, uploaded to every replica
    int rc = mbrwt_tree_parse(bytes, len, consumed, &t);
    if (rc) return rc;
    rc = mbrwt_multi_create(mbrwt_tree_get_desc(t), devices, n, out);
    mbrwt_tree_free(t);
    return rc;
}

void mbrwt_multi_destroy(mbrwt_multi *m) { destroy(m); }

int mbrwt_multi_size(const mbrwt_multi *m) { return m ? (int)m->ctx.size() : 0; }

mbrwt_ctx *mbrwt_multi_replica(mbrwt_multi *m, int i) {
    return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[i] : nullptr;
}

int mbrwt_multi_get_rows(mbrwt_multi *m, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                         uint64_t cols_cap, uint64_t *cols_needed) {
    if (!m || !offsets || (n && !rows)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    try {
        std::vector<uint64_t> need;
        int rc = run_slices(*m, rows, true, n, need, nullptr);
        if (rc) return rc;
        const uint32_t k = (uint32_t)m->ctx.size();
        std::vector<uint64_t> pre(k + 1, 0);
        for (uint32_t r = 0; r < k; ++r) pre[r + 1] = pre[r] + need[r];
        if (cols_needed) *cols_needed = pre[k];
        if (pre[k] > cols_cap || (pre[k] && !cols)) {
            set_error("cols_cap too small");
            return MBRWT_ERR_CAPACITY;
        }
        // each slice straight to its place: labels at the slice's label
        // offset, row offsets rebased on the host (one thread per replica)
        std::vector<int> st(k, MBRWT_OK);
        auto put = [&](uint32_t r) -> int {
            uint64_t lo, hi;
            slice(n, k, r, lo, hi);
            MBRWT_HIP(hipSetDevice(m->dev[r]));
            if (hi > lo)
                MBRWT_HIP(hipMemcpyAsync(offsets + lo, m->off[r].buf, (hi - lo) * 8, hipMemcpyDeviceToHost,
                                         m->stream[r]));
            if (need[r])
                MBRWT_HIP(hipMemcpyAsync(cols + pre[r], m->cols[r].buf, need[r] * 4, hipMemcpyDeviceToHost,
                                         m->stream[r]));
            MBRWT_HIP(hipStreamSynchronize(m->stream[r]));
            for (uint64_t i = lo; i < hi; ++i) offsets[i] += pre[r];
            return MBRWT_OK;
        };
        std::vector<std::thread> pool;
        for (uint32_t r = 1; r < k; ++r) pool.emplace_back([&, r]() { st[r] = put(r); });
        st[0] = put(0);
        for (auto &t : pool) t.join();
        for (uint32_t r = 0; r < k; ++r)
            if (st[r]) return st[r];
        offsets[n] = pre[k];
        return MBRWT_OK;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_multi_get_rows");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_multi_get_rows_device(mbrwt_multi *m, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                                uint32_t *d_cols, uint64_t cols_cap, uint64_t *cols_needed, void *stream) {
    if (!m || !d_offsets || (n && !d_rows)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    try {
        const hipStream_t s0 = reinterpret_cast<hipStream_t>(stream);
        std::vector<uint64_t> need;
        int rc = run_slices(*m, d_rows, false, n, need, s0);
        if (rc) return rc;
        const uint32_t k = (uint32_t)m->ctx.size();
        std::vector<uint64_t> pre(k + 1, 0);
        for (uint32_t r = 0; r < k; ++r) pre[r + 1] = pre[r] + need[r];
        if (cols_needed) *cols_needed = pre[k];
        if (pre[k] > cols_cap || (pre[k] && !d_cols)) {
            set_error("cols_cap too small");
            return MBRWT_ERR_CAPACITY;
        }
        // rebase each slice's offsets on its own device, then peer copies
        // into the caller's buffers on device 0 (xGMI; a plain copy for
        // replica 0), all ordered before the caller's stream continues
        for (uint32_t r = 0; r < k; ++r) {
            uint64_t lo, hi;
            slice(n, k, r, lo, hi);
            MBRWT_HIP(hipSetDevice(m->dev[r]));
            uint64_t *off = reinterpret_cast<uint64_t *>(m->off[r].buf);
            if (pre[r]) {
                const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((hi - lo + 256) / 256, 4096));
                hipLaunchKernelGGL(k_rebase, dim3((unsigned)g), dim3(256), 0, m->stream[r], off, hi - lo + 1, pre[r]);
                MBRWT_HIP(hipGetLastError());
            }
            MBRWT_HIP(hipMemcpyPeerAsync(d_offsets + lo, m->dev[0], off, m->dev[r], (hi - lo + (r + 1 == k)) * 8,
                                         m->stream[r]));
            if (need[r])
                MBRWT_HIP(hipMemcpyPeerAsync(d_cols + pre[r], m->dev[0], m->cols[r].buf, m->dev[r], need[r] * 4,
                                             m->stream[r]));
        }
        for (uint32_t r = 0; r < k; ++r) {
            MBRWT_HIP(hipSetDevice(m->dev[r]));
            MBRWT_HIP(hipStreamSynchronize(m->stream[r]));
        }
        MBRWT_HIP(hipSetDevice(m->dev[0]));
        if (n == 0) MBRWT_HIP(hipMemsetAsync(d_offsets, 0, 8, s0));
        return MBRWT_OK;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_multi_get_rows_device");
        return MBRWT_ERR_INVALID;
    }
}

}  // extern "C"
