// Host -> HBM staging for batches whose chunk bytes live in host memory (the
// reference fetches them into host Buffers: ByteGetter.get_sync /
// Store.get_ranges_sync, src/zarr/abc/store.py:474-539).  The pieces are
// packed into a pinned buffer by a persistent pool of host threads, window by
// window, and every window is handed to the DMA engine (hipMemcpyAsync on the
// caller's copy stream) by the thread that completes it -- so packing, PCIe
// transfer and the caller's planning all overlap, with no per-window work in
// Python.  A parallel host memcpy serves the way back (pinned result -> a
// caller's host array).
#include <emmintrin.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zarrhip.h"

namespace {

// A fixed pool: run(n, fn) calls fn(i) for i in [0, n) on the pool's threads
// (and the caller's), returning when all calls have finished.
class Pool {
   public:
    void run(int nthreads, const std::function<void(int)>& fn) {
        if (nthreads <= 1) {
            fn(0);
            return;
        }
        std::unique_lock<std::mutex> call_lock(call_mu_);  // one job at a time
        ensure(nthreads - 1);
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            want_ = nthreads - 1;
            started_ = 0;
            done_ = 0;
            ++epoch_;
        }
        cv_.notify_all();
        fn(nthreads - 1);  // the caller takes the last slot
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return done_ == want_; });
        job_ = nullptr;
    }

   private:
    void ensure(int n) {
        while ((int)threads_.size() < n) {
            threads_.emplace_back([this] { loop(); });
            threads_.back().detach();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return epoch_ != seen && job_ != nullptr && started_ < want_; });
            seen = epoch_;
            const int slot = started_++;
            const std::function<void(int)>* fn = job_;
            g.unlock();
            (*fn)(slot);
            g.lock();
            if (++done_ == want_) done_cv_.notify_one();
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> threads_;
    const std::function<void(int)>* job_ = nullptr;
    int want_ = 0, started_ = 0, done_ = 0;
    uint64_t epoch_ = 0;
};

Pool& pool() {
    static Pool* p = new Pool();  // never destroyed: detached workers outlive static teardown
    return *p;
}

// Host copies into page-locked windows (and back out of them): 1 = streaming
// (non-temporal) 16-byte stores, which skip the read-for-ownership of every
// destination line that a cached store pays -- the packed bytes are read next
// by the DMA engine, not by this core; 0 = memcpy.  zhip_set_tuning(
// ZHIP_TUNE_STAGE_COPY, v) selects (measurement arms).
static uint32_t g_copy_nt = 1;

static void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t n) {
    if (!g_copy_nt || n < 4096) {
        std::memcpy(dst, src, n);
        return;
    }
    const uint64_t head = (16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const uint64_t nb = n / 64u;
    for (uint64_t i = 0; i < nb; ++i, dst += 64, src += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 48), d);
    }
    std::memcpy(dst, src, n - nb * 64u);
    _mm_sfence();  // the streamed lines are visible (to the DMA engine) before the copy is enqueued
}

// Page-locked pieces: straight DMA, merged while both the host and the
// device sides stay contiguous (a pinned store's values lie in its arena in
// write order, with the same alignment gaps as the layout).  Returns whether
// any pageable piece is left for pack_windows; *rc is set on a HIP error.
static bool enqueue_pinned(const zhip_piece* pieces, uint32_t n_pieces, uint8_t* d, hipStream_t st, int* rc) {
    bool any_packed = false;
    for (uint32_t i = 0; i < n_pieces;) {
        if (!(pieces[i].flags & ZHIP_PIECE_PINNED) || pieces[i].nbytes == 0) {
            any_packed |= pieces[i].nbytes != 0;
            ++i;
            continue;
        }
        uint32_t j = i + 1;
        while (j < n_pieces && (pieces[j].flags & ZHIP_PIECE_PINNED) && pieces[j].nbytes &&
               pieces[j].host - pieces[i].host == pieces[j].dst_off - pieces[i].dst_off &&
               pieces[j].host >= pieces[j - 1].host + pieces[j - 1].nbytes &&
               pieces[j].host - (pieces[j - 1].host + pieces[j - 1].nbytes) < 256)
            ++j;
        const uint64_t n = pieces[j - 1].dst_off + pieces[j - 1].nbytes - pieces[i].dst_off;
        if (hipMemcpyAsync(d + pieces[i].dst_off, reinterpret_cast<const void*>(pieces[i].host), n,
                           hipMemcpyHostToDevice, st) != hipSuccess)
            *rc = ZHIP_E_HIP;
        i = j;
    }
    return any_packed;
}

// pread [off, off + n) of a file into dst; false unless every byte arrived
static bool read_file_range(const char* path, uint64_t off, uint8_t* dst, uint64_t n) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    bool ok = true;
    while (n > 0) {
        const ssize_t r = ::pread(fd, dst, n, (off_t)off);
        if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            ok = false;
            break;
        }
        dst += r;
        off += (uint64_t)r;
        n -= (uint64_t)r;
    }
    ::close(fd);
    return ok;
}

// A second, library-owned copy stream per device (ZHIP_TUNE_STAGE_STREAMS=2):
// windows alternate between the caller's stream and this one, so one DMA
// queue's per-copy gap could overlap the other's transfer.  Measured slower end
// to end (C2 from a MemoryStore: 2.17-2.34 ms vs 1.99-2.06 ms with one
// stream), so one stream is the default.
static hipStream_t aux_stream(hipStream_t st) {
    static std::mutex mu;
    static hipStream_t streams[64] = {};
    hipDevice_t dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!streams[dev]) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return nullptr;
        if (hipSetDevice(dev) != hipSuccess) return nullptr;
        if (hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking) != hipSuccess) streams[dev] = nullptr;
        (void)hipSetDevice(cur);
    }
    return streams[dev];
}

static uint32_t g_stage_streams = 1;  // zhip_set_tuning(ZHIP_TUNE_STAGE_STREAMS, n): 1 or 2

static int pack_windows(const zhip_piece* pieces, uint32_t n_pieces, uint8_t* pinned, uint8_t* d, uint64_t total,
                        uint64_t window, uint32_t nthreads, hipStream_t st) {
    std::atomic<int> rc{ZHIP_OK};
    if (window < 4096) window = 4096;
    // Pageable pieces: windows ramp up from window/16 (the first DMA starts
    // after a small pack, not a whole window) to `window`; one window per
    // task, taken in order, packed by one thread, which then enqueues the
    // window's packed runs.  (Packing a window by all threads together in
    // 256 KiB sub-ranges starts the first DMA sooner too but measured 30 %
    // slower end to end: scripts/stage_micro.py.)
    std::vector<uint64_t> edge{0};
    for (uint64_t w = window >= (64u << 10) ? window / 16 : window; edge.back() < total; w = w * 2 < window ? w * 2 : window)
        edge.push_back(edge.back() + w < total ? edge.back() + w : total);
    const uint64_t n_win = edge.size() - 1;
    // pieces are sorted by destination offset: window w starts at the first
    // piece reaching past its start
    std::vector<uint32_t> first(n_win + 1, n_pieces);
    {
        uint32_t i = 0;
        for (uint64_t w = 0; w < n_win; ++w) {
            while (i < n_pieces && pieces[i].dst_off + pieces[i].nbytes <= edge[w]) ++i;
            first[w] = i;
        }
    }
    // windows alternate between st and the aux stream, which first waits for
    // what st holds (the destination's earlier users) and is waited for by st
    // at the end (the consumer waits on st)
    hipStream_t qs[2] = {st, st};
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    if (g_stage_streams >= 2 && n_win >= 4) {
        hipStream_t aux = aux_stream(st);
        if (aux && hipEventCreateWithFlags(&ev_in, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&ev_out, hipEventDisableTiming) == hipSuccess &&
            hipEventRecord(ev_in, st) == hipSuccess && hipStreamWaitEvent(aux, ev_in, 0) == hipSuccess)
            qs[1] = aux;
    }
    std::atomic<uint64_t> next{0};
    auto worker = [&](int) {
        for (;;) {
            const uint64_t w = next.fetch_add(1);
            if (w >= n_win) return;
            const hipStream_t st = qs[w & 1];
            const uint64_t a = edge[w], b = edge[w + 1];
            uint64_t run_s = 0, run_e = 0;  // packed run (alignment pads between pieces ride along)
            auto flush = [&] {
                if (run_e > run_s &&
                    hipMemcpyAsync(d + run_s, pinned + run_s, run_e - run_s, hipMemcpyHostToDevice, st) != hipSuccess)
                    rc.store(ZHIP_E_HIP);
                run_s = run_e = 0;
            };
            for (uint32_t i = first[w]; i < n_pieces && pieces[i].dst_off < b; ++i) {
                const zhip_piece& pc = pieces[i];
                if (pc.flags & ZHIP_PIECE_PINNED) {
                    if (pc.nbytes) flush();
                    continue;
                }
                const uint64_t s = pc.dst_off > a ? pc.dst_off : a;
                const uint64_t e = pc.dst_off + pc.nbytes < b ? pc.dst_off + pc.nbytes : b;
                if (s >= e) continue;
                if (pc.flags & ZHIP_PIECE_FILE) {
                    if (!read_file_range(reinterpret_cast<const char*>(pc.host), pc.file_off + (s - pc.dst_off),
                                         pinned + s, e - s))
                        rc.store(ZHIP_E_IO);
                } else {
                    copy_bytes(pinned + s, reinterpret_cast<const uint8_t*>(pc.host) + (s - pc.dst_off), e - s);
                }
                if (run_e > run_s && s - run_e >= 256) flush();  // a real gap: leave it alone
                if (run_e == run_s) run_s = s;
                run_e = e;
            }
            flush();
        }
    };
    const uint32_t nt = nthreads == 0 ? 1u : (nthreads > 64 ? 64u : nthreads);
    pool().run((int)(nt < n_win ? nt : n_win), worker);
    if (qs[1] != st) {
        if (hipEventRecord(ev_out, qs[1]) != hipSuccess || hipStreamWaitEvent(st, ev_out, 0) != hipSuccess)
            rc.store(ZHIP_E_HIP);
    }
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    return rc.load();
}

}  // namespace

extern "C" {

int zhip_stage_h2d(const zhip_piece* pieces, uint32_t n_pieces, uint8_t* pinned, void* dev, uint64_t total,
                   uint64_t window, uint32_t nthreads, void* stream) {
    if (total == 0) return ZHIP_OK;
    if (!pinned || !dev || (!pieces && n_pieces)) return ZHIP_E_INVALID;
    int rc = ZHIP_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint8_t* const d = static_cast<uint8_t*>(dev);
    if (enqueue_pinned(pieces, n_pieces, d, st, &rc)) {
        const int r2 = pack_windows(pieces, n_pieces, pinned, d, total, window, nthreads, st);
        if (r2 != ZHIP_OK) rc = r2;
    }
    return rc;
}

// The same job started on a host thread of the library (no caller thread, no
// Python GIL needed while it runs); zhip_stage_end joins it.
// Staging jobs run in the order they were begun (a ticket each): a caller
// that begins several jobs at once (one per slab of a read) gets its slabs
// packed and copied in slab order.
static std::mutex g_job_mu;
static std::condition_variable g_job_cv;
static uint64_t g_job_next = 0, g_job_serving = 0;

struct zhip_stage_job {
    std::vector<zhip_piece> pieces;
    uint8_t* pinned;
    void* dev;
    uint64_t total, window;
    uint32_t nthreads;
    void* stream;
    int rc;
    hipEvent_t done;  // recorded on `stream` after the job's last copy
    std::thread th;
};

zhip_stage_job* zhip_stage_begin(const zhip_piece* pieces, uint32_t n_pieces, uint8_t* pinned, void* dev,
                                 uint64_t total, uint64_t window, uint32_t nthreads, void* stream) {
    zhip_stage_job* j = new (std::nothrow) zhip_stage_job();
    if (!j) return nullptr;
    j->rc = ZHIP_OK;
    j->done = nullptr;
    if (total == 0) return j;
    if (!pinned || !dev || (!pieces && n_pieces)) {
        j->rc = ZHIP_E_INVALID;
        return j;
    }
    if (hipEventCreateWithFlags(&j->done, hipEventDisableTiming) != hipSuccess) {
        j->done = nullptr;
        j->rc = ZHIP_E_HIP;
        return j;
    }
    // page-locked pieces: enqueued here, in the caller's order (a few
    // hipMemcpyAsync calls); a job with nothing to pack is complete now
    hipStream_t st0 = static_cast<hipStream_t>(stream);
    if (!enqueue_pinned(pieces, n_pieces, static_cast<uint8_t*>(dev), st0, &j->rc)) {
        if (hipEventRecord(j->done, st0) != hipSuccess) j->rc = ZHIP_E_HIP;
        return j;
    }
    j->pieces.assign(pieces, pieces + n_pieces);
    j->pinned = pinned;
    j->dev = dev;
    j->total = total;
    j->window = window;
    j->nthreads = nthreads;
    j->stream = stream;
    uint64_t ticket;
    {
        std::lock_guard<std::mutex> g(g_job_mu);
        ticket = g_job_next++;
    }
    j->th = std::thread([j, ticket] {
        {
            std::unique_lock<std::mutex> g(g_job_mu);
            g_job_cv.wait(g, [&] { return g_job_serving == ticket; });
        }
        hipStream_t st = static_cast<hipStream_t>(j->stream);
        int r = j->rc;
        const int r2 = pack_windows(j->pieces.data(), (uint32_t)j->pieces.size(), j->pinned,
                                    static_cast<uint8_t*>(j->dev), j->total, j->window, j->nthreads, st);
        if (r2 != ZHIP_OK) r = r2;
        // in ticket order: the event covers this job's windows and earlier
        // jobs' (and pinned copies already enqueued by later begins)
        if (hipEventRecord(j->done, st) != hipSuccess) r = ZHIP_E_HIP;
        j->rc = r;
        {
            std::lock_guard<std::mutex> g(g_job_mu);
            ++g_job_serving;
        }
        g_job_cv.notify_all();
    });
    return j;
}

// Events a stream was told to wait for are destroyed only once they have
// completed (checked at later stage_end calls), never right after the wait.
static std::mutex g_retire_mu;
static std::vector<hipEvent_t> g_retire;

static void retire_event(hipEvent_t ev) {
    std::lock_guard<std::mutex> g(g_retire_mu);
    g_retire.push_back(ev);
    size_t k = 0;
    for (size_t i = 0; i < g_retire.size(); ++i) {
        if (i + 1 < g_retire.size() && hipEventQuery(g_retire[i]) == hipSuccess)
            (void)hipEventDestroy(g_retire[i]);
        else
            g_retire[k++] = g_retire[i];
    }
    g_retire.resize(k);
}

int zhip_stage_end(zhip_stage_job* j, void* wait_stream) {
    if (!j) return ZHIP_E_INVALID;
    if (j->th.joinable()) j->th.join();
    int rc = j->rc;
    if (j->done) {
        // (wait_stream NULL is the default stream, which waits like any other)
        if (rc == ZHIP_OK && hipStreamWaitEvent(static_cast<hipStream_t>(wait_stream), j->done, 0) != hipSuccess)
            rc = ZHIP_E_HIP;
        retire_event(j->done);
    }
    delete j;
    return rc;
}

void zhip_stage_set_streams(uint32_t n) { g_stage_streams = n; }
void zhip_stage_set_copy(uint32_t nt) { g_copy_nt = nt ? 1u : 0u; }

int zhip_host_pinned(const void* p) {
    if (!p) return 0;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return 0;
    }
    return a.type == hipMemoryTypeHost ? 1 : 0;
}

int zhip_wait_words(const uint32_t* const* words, uint32_t n, uint32_t* host_out, void* stream) {
    // the per-call read's result check: each launch's 4-byte error word, read
    // back with one async copy per word into a page-locked per-thread buffer
    // behind the launches on `stream`, then one stream synchronise
    if (n == 0) return ZHIP_OK;
    if (!words || !host_out || n > 16) return ZHIP_E_INVALID;
    thread_local uint32_t* pinned = nullptr;
    if (!pinned && hipHostMalloc(reinterpret_cast<void**>(&pinned), 16 * sizeof(uint32_t), hipHostMallocDefault) !=
                       hipSuccess) {
        pinned = nullptr;
        return ZHIP_E_HIP;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    for (uint32_t i = 0; i < n; ++i)
        if (hipMemcpyAsync(pinned + i, words[i], sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
            return ZHIP_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return ZHIP_E_HIP;
    for (uint32_t i = 0; i < n; ++i) host_out[i] = pinned[i];
    return ZHIP_OK;
}

int zhip_wait_ranges(const void* const* srcs, const uint64_t* sizes, uint32_t n, void* host_out, void* stream) {
    // zhip_wait_words for ranges: every range copied back behind the launches
    // on `stream` into one page-locked per-thread buffer, one synchronise
    if (n == 0) return ZHIP_OK;
    if (!srcs || !sizes || !host_out) return ZHIP_E_INVALID;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += sizes[i];
    thread_local uint8_t* pinned = nullptr;
    thread_local uint64_t cap = 0;
    if (total > cap) {
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
        cap = 0;
        const uint64_t want = std::max<uint64_t>(total, 4096);
        if (hipHostMalloc(reinterpret_cast<void**>(&pinned), want, hipHostMallocDefault) != hipSuccess) {
            pinned = nullptr;
            return ZHIP_E_HIP;
        }
        cap = want;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (sizes[i] && hipMemcpyAsync(pinned + at, srcs[i], sizes[i], hipMemcpyDeviceToHost, st) != hipSuccess)
            return ZHIP_E_HIP;
        at += sizes[i];
    }
    if (hipStreamSynchronize(st) != hipSuccess) return ZHIP_E_HIP;
    std::memcpy(host_out, pinned, total);
    return ZHIP_OK;
}

int zhip_upload(const void* const* parts, const uint64_t* sizes, const uint64_t* offsets, uint32_t n, void* dev,
                uint64_t total, void* stream) {
    // a launch's host tables in one H2D copy: packed into a page-locked
    // per-thread, per-device buffer, whose previous copy (an event behind it)
    // has finished before it is overwritten
    if (total == 0) return ZHIP_OK;
    if (!dev || (n && (!parts || !sizes || !offsets))) return ZHIP_E_INVALID;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i] > total || sizes[i] > total - offsets[i] || (sizes[i] && !parts[i])) return ZHIP_E_INVALID;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return ZHIP_E_HIP;
    struct Slot {
        uint8_t* pinned = nullptr;
        uint64_t cap = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
    };
    thread_local Slot slots[64];
    Slot& s = slots[d];
    if (s.pending) {
        if (hipEventSynchronize(s.ev) != hipSuccess) return ZHIP_E_HIP;
        s.pending = false;
    }
    if (!s.ev && hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
        s.ev = nullptr;
        return ZHIP_E_HIP;
    }
    if (total > s.cap) {
        if (s.pinned) (void)hipHostFree(s.pinned);
        s.pinned = nullptr;
        s.cap = 0;
        uint64_t want = 1ull << 16;
        while (want < total) want <<= 1;
        if (hipHostMalloc(reinterpret_cast<void**>(&s.pinned), want, hipHostMallocDefault) != hipSuccess) {
            s.pinned = nullptr;
            return ZHIP_E_HIP;
        }
        s.cap = want;
    }
    for (uint32_t i = 0; i < n; ++i)
        if (sizes[i]) std::memcpy(s.pinned + offsets[i], parts[i], sizes[i]);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (hipMemcpyAsync(dev, s.pinned, total, hipMemcpyHostToDevice, st) != hipSuccess) return ZHIP_E_HIP;
    if (hipEventRecord(s.ev, st) != hipSuccess) return ZHIP_E_HIP;
    s.pending = true;
    return ZHIP_OK;
}

int zhip_host_copy(void* dst, const void* src, uint64_t nbytes, uint32_t nthreads) {
    if (nbytes == 0) return ZHIP_OK;
    if (!dst || !src) return ZHIP_E_INVALID;
    const uint64_t piece = 1ull << 20;
    const uint64_t n = (nbytes + piece - 1) / piece;
    std::atomic<uint64_t> next{0};
    auto worker = [&](int) {
        for (;;) {
            const uint64_t i = next.fetch_add(1);
            if (i >= n) return;
            const uint64_t a = i * piece, b = a + piece < nbytes ? a + piece : nbytes;
            // plain memcpy: the CPU reads the caller's array next, so the lines
            // stay cached (streaming stores serve the DMA packing direction)
            std::memcpy(static_cast<uint8_t*>(dst) + a, static_cast<const uint8_t*>(src) + a, b - a);
        }
    };
    const uint32_t nt = nthreads == 0 ? 1u : (nthreads > 64 ? 64u : nthreads);
    pool().run((int)(nt < n ? nt : n), worker);
    return ZHIP_OK;
}

}  // extern "C"
