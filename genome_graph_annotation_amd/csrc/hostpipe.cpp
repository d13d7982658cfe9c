// hostpipe.cpp -- the host-buffer get_rows (mbrwt_get_rows) as a chunked
// pipeline over PCIe.
//
// The reference's caller hands host vectors in and takes host vectors out
// (annotate_static.cpp:149-162 count_labels over get_row; main.cpp:462 one
// ThreadPool task per read batch).  On the device the batch costs ~45 ns per
// 1,000 rows; over PCIe the same batch moves 8 B per row in and 8 B + 4 B per
// label out, two orders of magnitude more time.  So the batch is cut into
// chunks of kChunkRows rows and the three transfers of consecutive chunks
// overlap: chunk i's row ids go up (stream `s_in`) while chunk i-1's labels
// come down (`s_out`) and the query of chunk i runs between them (the
// context's stream), each chunk in one of kSlots device slots.
//
// Host memory the runtime has page-locked (hipHostMalloc / hipHostRegister /
// torch pin_memory) is read and written by DMA directly.  Pageable memory is
// staged through pinned slot buffers: a pool of host threads copies chunk i+1's
// row ids in and chunk i-2's CSR out while the DMA engines move chunk i.
//
// Offsets: the device query writes chunk-local offsets; once the chunk's
// label count is known (its status block, read back as 3 u64), a small
// kernel adds the labels of the chunks before it, so the offsets land in the
// caller's buffer already global.  Capacity (include/mbrwt.h): the labels of
// a chunk are copied out only while the running total fits cols_cap; the
// counts continue, so *cols_needed is the batch's total either way.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "mbrwt_internal.hpp"

namespace mbrwt {

namespace {

constexpr uint64_t kChunkRows = 1ull << 20;  // 8 MiB of row ids, ~40 MiB of CSR at the Kingsford shape
constexpr int kSlots = 3;                    // chunk i in, i-1 out, i-2 copied to the caller

__global__ void k_add_base(uint64_t *off, uint64_t n, uint64_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) off[i] += base;
}

// a small pool of host threads for the pageable copies: run(f, parts) calls
// f(k) once for every k < parts (the caller takes parts too) and returns when
// all have run.  Parts are claimed under the mutex, tagged with the job's
// generation, so a worker still leaving one job never claims a part of the
// next with the previous function.
class CopyPool {
  public:
    explicit CopyPool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    void run(const std::function<void(unsigned)> &f, unsigned parts) {
        if (parts <= 1 || th_.empty()) {
            for (unsigned k = 0; k < parts; ++k) f(k);
            return;
        }
        uint64_t g;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            parts_ = parts;
            next_ = 0;
            left_ = parts;
            g = ++gen_;
        }
        cv_.notify_all();
        work(g);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    // claim and run parts of generation g until none is left
    void work(uint64_t g) {
        while (true) {
            const std::function<void(unsigned)> *f;
            unsigned k;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (gen_ != g || !job_ || next_ >= parts_) return;
                f = job_;
                k = next_++;
            }
            (*f)(k);
            std::lock_guard<std::mutex> lk(mu_);
            if (--left_ == 0) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        while (true) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work(seen);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)> *job_ = nullptr;
    unsigned parts_ = 0, next_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

void parallel_copy(CopyPool &pool, void *dst, const void *src, size_t bytes) {
    constexpr size_t kPiece = 4u << 20;
    const unsigned parts = (unsigned)std::min<size_t>(pool.size(), (bytes + kPiece - 1) / kPiece);
    if (parts <= 1) {
        if (bytes) std::memcpy(dst, src, bytes);
        return;
    }
    const size_t per = (bytes + parts - 1) / parts;
    pool.run(
        [&](unsigned k) {
            const size_t a = std::min(bytes, k * per), b = std::min(bytes, a + per);
            if (b > a) std::memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a);
        },
        parts);
}

bool is_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost || at.type == hipMemoryTypeManaged || at.type == hipMemoryTypeUnified;
}

}  // namespace

struct HostPipe {
    int device = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    struct Slot {
        Workspace rows, off, cols;                     // device
        uint64_t *h_status = nullptr;                  // pinned: the query's {labels, status, sticky}
        uint64_t *d_status = nullptr;
        void *h_rows = nullptr, *h_off = nullptr;      // pinned staging (pageable callers)
        void *h_cols = nullptr;
        size_t h_cols_bytes = 0;
        hipEvent_t ev_in = nullptr, ev_q = nullptr, ev_out = nullptr;
        uint64_t row0 = 0, n = 0, base = 0, need = 0;
        bool copy_cols = false;
    } slot[kSlots];
    CopyPool *pool = nullptr;
};

void free_host_pipe(HostPipe *p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    if (p->s_in) (void)hipStreamSynchronize(p->s_in);
    if (p->s_out) (void)hipStreamSynchronize(p->s_out);
    for (auto &s : p->slot) {
        for (Workspace *w : {&s.rows, &s.off, &s.cols})
            if (w->buf) (void)hipFree(w->buf);
        if (s.d_status) (void)hipFree(s.d_status);
        for (void *h : {(void *)s.h_status, s.h_rows, s.h_off, s.h_cols})
            if (h) (void)hipHostFree(h);
        for (hipEvent_t e : {s.ev_in, s.ev_q, s.ev_out})
            if (e) (void)hipEventDestroy(e);
    }
    if (p->s_in) (void)hipStreamDestroy(p->s_in);
    if (p->s_out) (void)hipStreamDestroy(p->s_out);
    delete p->pool;
    delete p;
}

static int pipe_init(Ctx &c) {
    if (c.pipe) return MBRWT_OK;
    HostPipe *p = new HostPipe();
    p->device = c.device;
    c.pipe = p;
    MBRWT_HIP(hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking));
    MBRWT_HIP(hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking));
    for (auto &s : p->slot) {
        MBRWT_HIP(hipHostMalloc(reinterpret_cast<void **>(&s.h_status), 4 * sizeof(uint64_t), hipHostMallocDefault));
        MBRWT_HIP(hipMalloc(&s.d_status, 4 * sizeof(uint64_t)));
        MBRWT_HIP(hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
        MBRWT_HIP(hipEventCreateWithFlags(&s.ev_q, hipEventDisableTiming));
        MBRWT_HIP(hipEventCreateWithFlags(&s.ev_out, hipEventDisableTiming));
        // (recorded once, so every wait on a slot's events has something to wait for)
        MBRWT_HIP(hipEventRecord(s.ev_out, p->s_out));
        MBRWT_HIP(hipEventRecord(s.ev_in, p->s_in));
        MBRWT_HIP(hipEventRecord(s.ev_q, p->s_in));
    }
    // copy threads beside the caller (r05: 15 instead of 7 changed nothing
    // measurable on the same box -- the pageable leg varies more between
    // boxes and runs than with the pool: profiles/r05/v13_copy_pool/)
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    p->pool = new CopyPool(std::min(7u, hw > 1 ? hw / 2 : 0u));
    return MBRWT_OK;
}

static int grow_pinned(void *&h, size_t &have, size_t bytes) {
    if (have >= bytes) return MBRWT_OK;
    if (h) MBRWT_HIP(hipHostFree(h));
    h = nullptr;
    have = 0;
    MBRWT_HIP(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    have = bytes;
    return MBRWT_OK;
}

// the query of one chunk on the context's stream: the asynchronous row-record
// call where it exists, else the synchronous call and its status block
static int enqueue_query(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_off, uint32_t *d_cols, uint64_t cap,
                         uint64_t *d_status, hipStream_t s) {
    MBRWT_HIP(hipMemsetAsync(d_status, 0, 3 * sizeof(uint64_t), s));
    if (c.rows.ready && c.kernel_variant == 0 && n > 0)
        return rows_get_rows(c, d_rows, n, d_off, d_cols, cap, nullptr, s, d_status);
    uint64_t need = 0;
    const int rc = run_get_rows(c, d_rows, n, d_off, d_cols, cap, &need, s);
    if (rc != MBRWT_OK && rc != MBRWT_ERR_CAPACITY && rc != MBRWT_ERR_RANGE) return rc;
    return rows_set_status(d_status, need, rc, s);
}

int host_get_rows(Ctx &c, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols, uint64_t cols_cap,
                  uint64_t *cols_needed) {
    int rc;
    if ((rc = pipe_init(c))) return rc;
    HostPipe &P = *c.pipe;
    const hipStream_t sq = c.stream;
    // every way out waits for the chunks already queued: an error return
    // (NOMEM growing a slot, a failed HIP call) must not leave H2D copies,
    // queries or D2H copies into the caller's page-locked buffers running
    // after the call has returned; on success the streams are
    // idle by then and the waits return at once
    struct Quiesce {
        HostPipe &P;
        hipStream_t sq;
        ~Quiesce() {
            (void)hipStreamSynchronize(P.s_in);
            (void)hipStreamSynchronize(sq);
            (void)hipStreamSynchronize(P.s_out);
        }
    } quiesce{P, sq};
    const bool pin_rows = is_pinned(rows), pin_off = is_pinned(offsets), pin_cols = cols && is_pinned(cols);
    const uint64_t nch = n ? (n + kChunkRows - 1) / kChunkRows : 1;
    const double mean = c.tree.num_rows ? (double)c.tree.num_relations / (double)c.tree.num_rows : 0.0;
    uint64_t total = 0;      // labels of the chunks drained so far
    int err = MBRWT_OK;      // first failing status (RANGE / DEVICE)
    uint64_t issued = 0;     // chunks queued (none after a failure)

    auto slot_of = [&](uint64_t i) -> HostPipe::Slot & { return P.slot[i % kSlots]; };

    // step 1: chunk i's row ids to the device, its query queued
    auto issue = [&](uint64_t i) -> int {
        HostPipe::Slot &s = slot_of(i);
        if (c.test_fail_chunk >= 0 && i == (uint64_t)c.test_fail_chunk) {  // (test hook: an injected NOMEM)
            set_error("injected failure (MBRWT_OPT_TEST_FAIL_CHUNK)");
            return MBRWT_ERR_NOMEM;
        }
        s.row0 = i * kChunkRows;
        s.n = std::min<uint64_t>(kChunkRows, n - s.row0);
        const uint64_t lcap = (uint64_t)((double)s.n * mean * 1.25) + 65536;
        int r;
        if ((r = ensure(s.rows, std::max<uint64_t>(1, s.n) * 8)) || (r = ensure(s.off, (s.n + 1) * 8)) ||
            (r = ensure(s.cols, lcap * 4)))
            return r;
        const uint64_t *src = rows + s.row0;
        if (!pin_rows && s.n) {
            // the staging slot is free once its previous H2D has run
            MBRWT_HIP(hipEventSynchronize(s.ev_in));
            size_t have = s.h_rows ? kChunkRows * 8 : 0;
            if ((r = grow_pinned(s.h_rows, have, kChunkRows * 8))) return r;
            parallel_copy(*P.pool, s.h_rows, src, s.n * 8);
            src = static_cast<const uint64_t *>(s.h_rows);
        }
        // the device slot is free once the chunk kSlots earlier has left it
        MBRWT_HIP(hipStreamWaitEvent(P.s_in, s.ev_q, 0));
        if (s.n) MBRWT_HIP(hipMemcpyAsync(s.rows.buf, src, s.n * 8, hipMemcpyHostToDevice, P.s_in));
        MBRWT_HIP(hipEventRecord(s.ev_in, P.s_in));
        MBRWT_HIP(hipStreamWaitEvent(sq, s.ev_in, 0));
        MBRWT_HIP(hipStreamWaitEvent(sq, s.ev_out, 0));
        if ((r = enqueue_query(c, static_cast<uint64_t *>(s.rows.buf), s.n, static_cast<uint64_t *>(s.off.buf),
                               static_cast<uint32_t *>(s.cols.buf), s.cols.bytes / 4, s.d_status, sq)))
            return r;
        MBRWT_HIP(hipMemcpyAsync(s.h_status, s.d_status, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, sq));
        MBRWT_HIP(hipEventRecord(s.ev_q, sq));
        return MBRWT_OK;
    };

    // step 2: chunk i's CSR leaves the device (its label count read first)
    auto drain = [&](uint64_t i) -> int {
        HostPipe::Slot &s = slot_of(i);
        MBRWT_HIP(hipEventSynchronize(s.ev_q));
        uint64_t need = s.h_status[0], st = s.h_status[1];
        if (st == MBRWT_ERR_CAPACITY) {  // a chunk denser than the slot's estimate: again, with room
            int r;
            if ((r = ensure(s.cols, need * 4 + 4096))) return r;
            if ((r = enqueue_query(c, static_cast<uint64_t *>(s.rows.buf), s.n, static_cast<uint64_t *>(s.off.buf),
                                   static_cast<uint32_t *>(s.cols.buf), s.cols.bytes / 4, s.d_status, sq)))
                return r;
            MBRWT_HIP(hipMemcpyAsync(s.h_status, s.d_status, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, sq));
            MBRWT_HIP(hipEventRecord(s.ev_q, sq));
            MBRWT_HIP(hipEventSynchronize(s.ev_q));
            need = s.h_status[0];
            st = s.h_status[1];
        }
        if (st != MBRWT_OK) {
            if (!err) err = (int)st;
            MBRWT_HIP(hipEventRecord(s.ev_out, P.s_out));
            s.copy_cols = false;
            s.need = 0;
            return MBRWT_OK;
        }
        s.base = total;
        s.need = need;
        total += need;
        s.copy_cols = cols && total <= cols_cap;
        if (err) {  // (no more output once a chunk has failed)
            MBRWT_HIP(hipEventRecord(s.ev_out, P.s_out));
            return MBRWT_OK;
        }
        MBRWT_HIP(hipStreamWaitEvent(P.s_out, s.ev_q, 0));
        uint64_t *doff = static_cast<uint64_t *>(s.off.buf);
        if (s.base && s.n)
            hipLaunchKernelGGL(k_add_base, dim3((unsigned)((s.n + 1 + 255) / 256)), dim3(256), 0, P.s_out, doff,
                               s.n + 1, s.base);
        MBRWT_HIP(hipGetLastError());
        // offsets[row0 .. row0 + n]: the last entry is the next chunk's first (equal values)
        const uint64_t last = (i + 1 == nch) ? 1 : 0;
        const size_t off_bytes = (s.n + last) * 8;
        if (pin_off) {
            if (off_bytes)
                MBRWT_HIP(hipMemcpyAsync(offsets + s.row0, doff, off_bytes, hipMemcpyDeviceToHost, P.s_out));
        } else if (off_bytes) {
            size_t have = s.h_off ? (kChunkRows + 1) * 8 : 0;
            int r;
            if ((r = grow_pinned(s.h_off, have, (kChunkRows + 1) * 8))) return r;
            MBRWT_HIP(hipMemcpyAsync(s.h_off, doff, off_bytes, hipMemcpyDeviceToHost, P.s_out));
        }
        if (s.copy_cols && need) {
            if (pin_cols) {
                MBRWT_HIP(hipMemcpyAsync(cols + s.base, s.cols.buf, need * 4, hipMemcpyDeviceToHost, P.s_out));
            } else {
                int r;
                if ((r = grow_pinned(s.h_cols, s.h_cols_bytes, need * 4))) return r;
                MBRWT_HIP(hipMemcpyAsync(s.h_cols, s.cols.buf, need * 4, hipMemcpyDeviceToHost, P.s_out));
            }
        }
        MBRWT_HIP(hipEventRecord(s.ev_out, P.s_out));
        return MBRWT_OK;
    };

    // step 3: a pageable caller's share of chunk i, from the staging slots
    auto finish = [&](uint64_t i) -> int {
        HostPipe::Slot &s = slot_of(i);
        if (err || (pin_off && (pin_cols || !s.copy_cols))) return MBRWT_OK;
        MBRWT_HIP(hipEventSynchronize(s.ev_out));
        const uint64_t last = (i + 1 == nch) ? 1 : 0;
        if (!pin_off && s.n + last) parallel_copy(*P.pool, offsets + s.row0, s.h_off, (s.n + last) * 8);
        if (s.copy_cols && !pin_cols && s.need) {
            parallel_copy(*P.pool, cols + s.base, s.h_cols, s.need * 4);
        }
        return MBRWT_OK;
    };

    if (n == 0) {
        offsets[0] = 0;
        if (cols_needed) *cols_needed = 0;
        return MBRWT_OK;
    }
    for (uint64_t i = 0; i < nch + 2; ++i) {
        if (i < nch && !err) {
            if ((rc = issue(i))) return rc;
            issued = i + 1;
        }
        if (i >= 1 && i - 1 < issued && (rc = drain(i - 1))) return rc;
        if (i >= 2 && i - 2 < issued && (rc = finish(i - 2))) return rc;
    }
    MBRWT_HIP(hipStreamSynchronize(P.s_out));
    MBRWT_HIP(hipStreamSynchronize(sq));
    if (cols_needed) *cols_needed = total;
    if (err == MBRWT_ERR_RANGE) {
        set_error("row out of range");
        return MBRWT_ERR_RANGE;
    }
    if (err) {
        set_error("row-record walk failed (corrupt image)");
        return MBRWT_ERR_DEVICE;
    }
    if (total > cols_cap || (!cols && total)) {
        set_error("cols_cap too small");
        return MBRWT_ERR_CAPACITY;
    }
    return MBRWT_OK;
}

}  // namespace mbrwt
