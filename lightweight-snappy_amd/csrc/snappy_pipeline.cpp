// snappy_pipeline.cpp -- host C++ built on the device shim (snappy_device.hip,
// through snappy_ctx.h): pooled per-thread host contexts, the host-buffer
// compress pipeline, the streaming FILE* compressor and decoder (positional
// multi-threaded I/O, mapped outputs, writer threads) and the calls over
// several devices.  No kernel is launched here: every GPU step goes through
// compress_impl / snappy_amd_*_device / snappy_amd_index_device and HIP
// runtime copies.  Declared in include/snappy_amd_internal.h (host-buffer
// and FILE* entry points used by snappy_host.c) and include/snappy_amd.h
// (host device selection, pool, *_multi).
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <fcntl.h>
#include <memory>
#include <mutex>
#include <new>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <time.h>
#include <unistd.h>
#include <vector>

#include "snappy_amd.h"
#include "snappy_amd_internal.h"
#include "snappy_ctx.h"

extern "C" {

// ---- host-buffer and FILE* paths (used by snappy_host.c) -------------------
//
// Streaming FILE* compress: the reference's fread/compress/
// fwrite block loop (snappy_compression.c:419-425) as a two-slot pipeline of
// 64 MiB chunks (a multiple of the 65,536-byte block, so block boundaries and
// bytes are those of the whole-input stream).  Slot k%2 has its own context
// (stream), pinned staging and device buffers: while chunk k's H2D + kernels
// run, the host writes chunk k-1 (exact-size D2H on the other stream) and
// reads chunk k+1.  Chunk 0 carries the varint(header_value) preamble, the
// others are compressed with it suppressed.
namespace {
// a host pipeline's context: its own stream made at once (the pipelines copy on
// c->stream before the first launch; device-API contexts create theirs lazily)
int create_host_ctx(int device, snappy_amd_ctx **out)
{
    int rc = snappy_amd_create(device, out);
    if (rc) return rc;
    if ((rc = ctx_stream(*out))) {
        snappy_amd_destroy(*out);
        *out = nullptr;
    }
    return rc;
}

// A pipeline context's own stream at high priority: high-priority streams take
// hardware queues of their own, where default-priority streams share the
// process's few (GPU_MAX_HW_QUEUES, 4 by default) with the caller's streams,
// and a stream sharing a queue waits behind the other's work (in bench.py's
// process, next to torch's streams, two host-pipeline lanes each shared a
// queue with another and the pipeline ran two chunks at a time: 256 MiB of
// text 21.9 -> 28.9 GB/s, profiles/r04n_*).  A failure keeps the stream.
void high_priority_stream(snappy_amd_ctx *c)
{
    int lo = 0, hi = 0;
    hipStream_t st = nullptr;
    if (c->stream != c->own || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&st, hipStreamDefault, hi) != hipSuccess)
        return;
    (void)hipStreamDestroy(c->own);
    c->own = c->stream = st;
}

struct StreamSlot {
    snappy_amd_ctx *c = nullptr;
    uint8_t *h_in = nullptr, *h_out = nullptr;
    uint64_t *h_idx = nullptr;  // the chunk's block index, for the sidecar file
    uint8_t *d_in = nullptr, *d_out = nullptr;
    uint64_t *d_idx = nullptr;
    size_t n = 0;
    bool busy = false;
};
constexpr size_t kStreamChunk = (size_t)64 << 20;

size_t read_full(FILE *f, uint8_t *b, size_t cap)
{
    size_t n = 0;
    while (n < cap) {
        const size_t got = fread(b + n, 1, cap - n, f);
        if (got == 0) break;
        n += got;
    }
    return n;
}

// SNAPPY_AMD_IO_TRACE=1: phase times of the FILE* pipelines on stderr
double io_now()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}
bool io_trace()
{
    static const bool on = getenv("SNAPPY_AMD_IO_TRACE") != nullptr;  // read once
    return on;
}

// Threads copying file chunks between the page cache and pinned staging:
// readers SNAPPY_AMD_IO_THREADS (default 8: one thread moves a few GB/s, the
// GPU path tens); writers SNAPPY_AMD_IO_WTHREADS (default 1: Linux serialises
// writes to one file on its inode lock, so more writers only contend --
// tools/io_probe.py on the GPU box's tmpfs: 5.8 GB/s with one, 3.6 with 8)
static int env_threads(const char *name, int dflt)
{
    int t = dflt;
    if (const char *e = getenv(name)) t = atoi(e);
    return t < 1 ? 1 : (t > 64 ? 64 : t);
}
int io_threads()
{
    static const int t = env_threads("SNAPPY_AMD_IO_THREADS", 8);
    return t;
}
int io_wthreads()
{
    static const int t = env_threads("SNAPPY_AMD_IO_WTHREADS", 1);
    return t;
}

// pread/pwrite of [off, off + len) split over io_threads() / io_wthreads()
// threads in 1 MiB aligned parts; returns the bytes moved (short only at EOF
// or on error)
size_t par_io(int fd, uint8_t *buf, size_t len, uint64_t off, bool wr)
{
    const int nt = len >= ((size_t)4 << 20) ? (wr ? io_wthreads() : io_threads()) : 1;
    const size_t per = ((len / nt) + (1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
    std::vector<size_t> done(nt, 0);
    auto part = [&](int t) {
        const size_t a = std::min(len, per * t), b = std::min(len, per * (t + 1));
        size_t x = a;
        while (x < b) {
            const ssize_t r = wr ? pwrite(fd, buf + x, b - x, (off_t)(off + x)) : pread(fd, buf + x, b - x, (off_t)(off + x));
            if (r <= 0) break;
            x += (size_t)r;
        }
        done[t] = x - a;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(part, t);
    part(0);
    for (auto &x : th) x.join();
    size_t tot = 0;  // the contiguous prefix moved (a short part ends it)
    for (int t = 0; t < nt; t++) {
        const size_t a = std::min(len, per * t), b = std::min(len, per * (t + 1));
        tot += done[t];
        if (done[t] != b - a) break;
    }
    return tot;
}

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif
// memcpy of len bytes into a shared file mapping, split over io_threads()
// threads in 1 MiB aligned parts; each thread first maps its part's pages
// writable in one call (MADV_POPULATE_WRITE; on older kernels the copy
// faults them in)
void par_copy(uint8_t *dst, const uint8_t *src, size_t len)
{
    const int nt = len >= ((size_t)4 << 20) ? io_threads() : 1;
    const size_t per = ((len / nt) + (1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    auto part = [&](int t) {
        const size_t a = std::min(len, per * t), b = std::min(len, per * (t + 1));
        if (b <= a) return;
        const uintptr_t lo = (uintptr_t)(dst + a) & ~(pg - 1), hi = (uintptr_t)(dst + b);
        (void)madvise((void *)lo, hi - lo, MADV_POPULATE_WRITE);
        memcpy(dst + a, src + a, b - a);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(part, t);
    part(0);
    for (auto &x : th) x.join();
}

// A FILE* used from its current position: positional multi-threaded I/O on a
// regular file (the stdio buffer is flushed / skipped; finish() leaves the
// FILE* where the stdio calls would have), plain fread / fwrite otherwise
// (pipes, terminals, files opened for append).
//
// A positional writer that knows a bound on what it will write can map the
// file instead (map_out): the output is then copied into the file's pages by
// io_threads() threads.  write() / pwrite() of one file serialise on its inode
// lock (one writer moved 5.9-10.5 GB/s into the GPU box's tmpfs, 8 were
// slower), faults on distinct pages of a shared mapping do not.  The file is
// extended to the bound while mapped and cut back to max(its old size, the
// bytes written) by finish() (or by the destructor on an error path);
// SNAPPY_AMD_NO_MMAP=1 keeps pwrite().
// Unmapping a large populated output mapping tears down its page tables
// (≈ 0.2 s for 4 GiB on the GPU box), after the file's bytes and size are
// final: a successful mapped writer hands the munmap (and the close of its
// read-write descriptor) to a background thread instead of waiting for it.
// Pending unmaps are joined by the next one queued and at exit.
// SNAPPY_AMD_SYNC_UNMAP=1 unmaps in the call.
struct UnmapReaper {
    struct Job {
        void *map;
        size_t len;
        int close_fd;
    };
    std::mutex mu;
    std::vector<pthread_t> ts;  // (raw ids: a forked child forgets its parent's, see below)
    static void *run(void *a)
    {
        const Job *j = static_cast<Job *>(a);
        (void)munmap(j->map, j->len);
        if (j->close_fd >= 0) ::close(j->close_fd);
        delete j;
        return nullptr;
    }
    UnmapReaper()
    {
        // a child forked while an unmap runs has no such thread: it must not join it at exit
        (void)pthread_atfork(nullptr, nullptr, [] { g_reaper_forget(); });
    }
    static void g_reaper_forget();
    void queue(void *map, size_t len, int close_fd)
    {
        Job *j = new Job{map, len, close_fd};
        std::vector<pthread_t> done;
        pthread_t t;
        std::lock_guard<std::mutex> lk(mu);
        done.swap(ts);
        if (pthread_create(&t, nullptr, run, j) == 0) ts.push_back(t);
        else run(j);  // no thread: unmap here
        for (pthread_t d : done) pthread_join(d, nullptr);
    }
    ~UnmapReaper()
    {
        std::lock_guard<std::mutex> lk(mu);
        for (pthread_t t : ts) pthread_join(t, nullptr);
        ts.clear();
    }
};
UnmapReaper g_reaper;
void UnmapReaper::g_reaper_forget()  // (the child is single-threaded: a lock held at fork is reset)
{
    new (&g_reaper.mu) std::mutex();
    g_reaper.ts.clear();
}
bool async_unmap()
{
    static const bool a = [] {
        const char *e = getenv("SNAPPY_AMD_SYNC_UNMAP");
        return !(e && atoi(e) != 0);
    }();
    return a;
}

struct IoFile {
    FILE *f = nullptr;
    int fd = -1;
    bool pos_io = false;
    uint64_t pos = 0;
    uint8_t *map = nullptr;
    size_t map_len = 0;
    uint64_t map_at = 0, map_end = 0, old_size = 0, map_from = 0;
    int map_fd = -1;
    IoFile() = default;
    IoFile(const IoFile &) = delete;
    IoFile &operator=(const IoFile &) = delete;
    ~IoFile() { unmap(); }
    bool open(FILE *file, bool wr)
    {
        f = file;
        if (wr && fflush(f) != 0) return false;
        fd = fileno(f);
        struct stat st;
        const off_t p = ftello(f);
        pos_io = fd >= 0 && p >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) &&
                 !(wr && (fcntl(fd, F_GETFL) & O_APPEND));
        pos = pos_io ? (uint64_t)p : 0;
        return true;
    }
    uint64_t remaining() const  // bytes to EOF (positional readers only)
    {
        struct stat st;
        if (!pos_io || fstat(fd, &st) != 0) return 0;
        return (uint64_t)st.st_size > pos ? (uint64_t)st.st_size - pos : 0;
    }
    // map [pos, pos + bound) for writing; false (nothing changed) if this file
    // cannot be mapped: the caller keeps pwrite()
    bool map_out(uint64_t bound)
    {
        if (!pos_io || map || bound < ((uint64_t)64 << 20) || getenv("SNAPPY_AMD_NO_MMAP")) return false;
        int rfd = fd;
        if ((fcntl(fd, F_GETFL) & O_ACCMODE) != O_RDWR) {  // a shared mapping needs a read-write descriptor
            char path[64];
            snprintf(path, sizeof path, "/proc/self/fd/%d", fd);
            rfd = ::open(path, O_RDWR | O_CLOEXEC);
            if (rfd < 0) return false;
        }
        struct stat st;
        const uint64_t end = pos + bound;
        const long pg = sysconf(_SC_PAGESIZE);
        bool ok = fstat(rfd, &st) == 0 && S_ISREG(st.st_mode) && pg > 0;
        if (ok) {
            old_size = (uint64_t)st.st_size;
            ok = old_size >= end || ftruncate(rfd, (off_t)end) == 0;
        }
        void *m = MAP_FAILED;
        if (ok) {
            map_at = pos & ~(uint64_t)(pg - 1);
            map_len = (size_t)(end - map_at);
            m = mmap(nullptr, map_len, PROT_READ | PROT_WRITE, MAP_SHARED, rfd, (off_t)map_at);
        }
        if (m == MAP_FAILED) {
            if (ok && old_size < end) (void)ftruncate(rfd, (off_t)old_size);
            if (rfd != fd) ::close(rfd);
            return false;
        }
        map = static_cast<uint8_t *>(m);
        map_fd = rfd;
        map_end = end;
        map_from = pos;
        return true;
    }
    // unmap; the file keeps max(its old size, the end of the bytes written) --
    // its old size if nothing was written (an error before the first chunk)
    bool unmap(bool background = false)
    {
        if (!map) return true;
        const uint64_t keep = pos > map_from ? std::max(old_size, pos) : old_size;
        bool ok = true;
        if (background && map_end <= keep && async_unmap()) {  // nothing to cut back: bytes and size are final
            g_reaper.queue(map, map_len, map_fd != fd ? map_fd : -1);
        } else {
            ok = munmap(map, map_len) == 0;
            if (map_end > keep) ok = ftruncate(map_fd, (off_t)keep) == 0 && ok;
            if (map_fd != fd) ::close(map_fd);
        }
        map = nullptr;
        map_fd = -1;
        return ok;
    }
    size_t read(uint8_t *b, size_t cap)
    {
        if (!pos_io) return read_full(f, b, cap);
        const size_t got = par_io(fd, b, cap, pos, false);
        pos += got;
        return got;
    }
    bool write(const uint8_t *b, size_t len)
    {
        if (!len) return true;
        if (map) {
            if (pos + len > map_end) return false;
            par_copy(map + (pos - map_at), b, len);
            pos += len;
            return true;
        }
        if (!pos_io) return fwrite(b, 1, len, f) == len;
        const size_t put = par_io(fd, const_cast<uint8_t *>(b), len, pos, true);
        pos += put;
        return put == len;
    }
    bool error() const { return !pos_io && ferror(f); }
    bool finish() { return unmap(true) && (!pos_io || fseeko(f, (off_t)pos, SEEK_SET) == 0); }
};

void slot_free(StreamSlot &s)
{
    for (void *h : {(void *)s.h_in, (void *)s.h_out, (void *)s.h_idx})
        if (h) (void)hipHostFree(h);
    for (void *d : {(void *)s.d_in, (void *)s.d_out, (void *)s.d_idx})
        if (d) (void)hipFree(d);
    snappy_amd_destroy(s.c);
    s = StreamSlot{};
}

// a slot is usable only when every buffer exists: a partial failure frees
// what was allocated, so the next call retries from scratch
int slot_init(StreamSlot &s, int device)
{
    if (s.c) return SNAPPY_AMD_OK;
    int rc = create_host_ctx(device, &s.c);
    if (rc) return rc;
    const size_t maxo = snappy_amd_max_output(kStreamChunk, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE);
    const size_t units = kStreamChunk / SNAPPY_AMD_BLOCK;
    if (hipHostMalloc(&s.h_in, kStreamChunk, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_out, maxo, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_idx, (units + 1) * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s.d_in, kStreamChunk) != hipSuccess || hipMalloc(&s.d_out, maxo) != hipSuccess ||
        hipMalloc(&s.d_idx, (units + 1) * sizeof(uint64_t)) != hipSuccess) {
        slot_free(s);
        return SNAPPY_AMD_ERR_DEVICE;
    }
    return SNAPPY_AMD_OK;
}

// The compressed chunks go to the file from a writer thread, one chunk at a
// time and in order, so writing chunk k-1 overlaps reading chunk k+1 (the two
// use different buffers of the slot); wait() joins the chunk in flight.
struct AsyncWriter {
    std::thread t;
    bool ok = true;
    double busy = 0;  // seconds spent writing (SNAPPY_AMD_IO_TRACE)
    void wait()
    {
        if (t.joinable()) t.join();
    }
    // false if an earlier chunk failed to write (nothing more is written)
    bool start(IoFile &f, const uint8_t *b, size_t len)
    {
        wait();
        if (!ok) return false;
        t = std::thread([this, &f, b, len] {
            const double t0 = io_now();
            ok = f.write(b, len);
            busy += io_now() - t0;
        });
        return true;
    }
    ~AsyncWriter() { wait(); }
};

// finish slot s: its compressed size is in s.c->h_total once its stream drains.
// With a sidecar file, the chunk's block index goes out too, shifted by the
// stream bytes written before it (*base); the stream-end entry is left to the caller.
// The chunk's bytes are handed to the writer (the slot's h_out stays in use
// until the next drain's start() joins it: the slots alternate, so that is
// two drains before this slot's h_out is filled again).
int slot_drain(StreamSlot &s, AsyncWriter &wr, IoFile &fout, FILE *fidx, uint64_t *base)
{
    if (!s.busy) return SNAPPY_AMD_OK;
    s.busy = false;
    HIP_OK(hipStreamSynchronize(s.c->stream));
    const size_t len = (size_t)*s.c->h_total;
    const size_t units = (s.n + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    HIP_OK(hipMemcpyAsync(s.h_out, s.d_out, len, hipMemcpyDeviceToHost, s.c->stream));
    if (fidx) HIP_OK(hipMemcpyAsync(s.h_idx, s.d_idx, units * sizeof(uint64_t), hipMemcpyDeviceToHost, s.c->stream));
    HIP_OK(hipStreamSynchronize(s.c->stream));
    if (!wr.start(fout, s.h_out, len)) return SNAPPY_AMD_ERR_IO;
    if (fidx) {
        for (size_t i = 0; i < units; i++) s.h_idx[i] += *base;
        if (fwrite(s.h_idx, sizeof(uint64_t), units, fidx) != units) return SNAPPY_AMD_ERR_IO;
    }
    *base += len;
    return SNAPPY_AMD_OK;
}

// pinned staging of the FILE* decoder: 3 chunks in rotation (one being
// filled or drained by the host threads while the copy engine moves another)
struct DecStage {
    uint8_t *h[3] = {};
    hipEvent_t ev[3] = {};
    bool ready = false;
};

void dec_stage_free(DecStage &d)
{
    for (int j = 0; j < 3; j++) {
        if (d.h[j]) (void)hipHostFree(d.h[j]);
        if (d.ev[j]) (void)hipEventDestroy(d.ev[j]);
        d.h[j] = nullptr;
        d.ev[j] = nullptr;
    }
    d.ready = false;
}

int dec_stage_init(DecStage &d)
{
    if (d.ready) return SNAPPY_AMD_OK;
    for (int i = 0; i < 3; i++) {
        if (hipHostMalloc(&d.h[i], kStreamChunk, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&d.ev[i], hipEventDisableTiming) != hipSuccess) {
            dec_stage_free(d);
            return SNAPPY_AMD_ERR_DEVICE;
        }
    }
    d.ready = true;
    return SNAPPY_AMD_OK;
}

// Host calls (host-buffer and FILE* APIs) run on pooled host contexts: a call
// leases an idle context of its device (or creates one) and returns it at the
// end, so concurrent calls from several threads run concurrently, each on its
// own streams, scratch and pinned staging.  The pool's lock is held only to
// take or return a context.  The device is the calling thread's
// (snappy_amd_host_set_device), else SNAPPY_AMD_DEVICE (read once), else 0.
constexpr int kPipeLanesMax = 16;
// host-buffer compress: chunks in flight (SNAPPY_AMD_PIPE_LANES, default 4) of
// SNAPPY_AMD_PIPE_CHUNK_MB MiB each (a multiple of the 65,536-byte block; default 64 = 1,024 blocks)
int pipe_lanes()
{
    static const int l = std::min(kPipeLanesMax, env_threads("SNAPPY_AMD_PIPE_LANES", 4));
    return l;
}
size_t pipe_chunk()
{
    static const size_t c = (size_t)std::max(1, std::min(4096, env_threads("SNAPPY_AMD_PIPE_CHUNK_MB", 64))) << 20;
    return c;
}

struct HostCtx {
    int device = 0;
    snappy_amd_ctx *c = nullptr;           // host-buffer path and the FILE* decoder
    StreamSlot slots[2];                   // the FILE* compressor's two pipeline slots
    DecStage dec;                          // the FILE* decoder's pinned staging
    snappy_amd_ctx *pipe[kPipeLanesMax] = {}; // the host-buffer compressor's chunk lanes
};

void host_free(HostCtx *h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (auto &s : h->slots) slot_free(s);
    for (auto *p : h->pipe)
        if (p != h->c) snappy_amd_destroy(p);
    dec_stage_free(h->dec);
    snappy_amd_destroy(h->c);
    delete h;
}

std::mutex g_pool_mu;
std::vector<HostCtx *> g_pool;  // idle host contexts, any device
thread_local int t_host_device = -1;

int default_device()
{
    static const int d = [] {
        const char *e = getenv("SNAPPY_AMD_DEVICE");
        return e ? atoi(e) : 0;
    }();
    return d;
}

int host_device() { return t_host_device >= 0 ? t_host_device : default_device(); }

class Lease {
public:
    explicit Lease(int device)
    {
        {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            for (size_t i = g_pool.size(); i-- > 0;)
                if (g_pool[i]->device == device) {
                    h_ = g_pool[i];
                    g_pool.erase(g_pool.begin() + (long)i);
                    break;
                }
        }
        if (!h_) {
            HostCtx *h = new HostCtx();
            h->device = device;
            rc_ = create_host_ctx(device, &h->c);
            if (rc_) delete h;
            else h_ = h;
        }
        if (h_ && hipSetDevice(device) != hipSuccess) rc_ = SNAPPY_AMD_ERR_DEVICE;
    }
    ~Lease()
    {
        if (!h_) return;
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool.push_back(h_);
    }
    Lease(const Lease &) = delete;
    Lease &operator=(const Lease &) = delete;
    int rc() const { return rc_; }
    HostCtx &operator*() const { return *h_; }
    HostCtx *operator->() const { return h_; }

private:
    HostCtx *h_ = nullptr;
    int rc_ = SNAPPY_AMD_OK;
};

// one SINGLE-layout stream (or, with NO_PREAMBLE, a block-aligned part of
// one) of in[0..n) on host context h: H2D, kernels, the compressed bytes left
// in h.c->d_b and the block index in h.c->d_idx; *len = compressed bytes
int host_compress_stage(HostCtx &h, const uint8_t *in, size_t n, uint32_t flags, uint64_t header_value, size_t *len)
{
    snappy_amd_ctx *c = h.c;
    const size_t units = (n + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    const size_t maxo = snappy_amd_max_output(n, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE);
    int rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_a), &c->d_a_cap, n + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_b), &c->d_b_cap, maxo))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap, (units + 1) * sizeof(uint64_t)))) return rc;
    HIP_OK(hipMemcpyAsync(c->d_a, in, n, hipMemcpyHostToDevice, c->stream));
    return compress_impl(c, c->d_a, n, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, flags, header_value, c->d_b, c->d_idx, len);
}

// a sidecar index's shape: one entry per block + the end, every entry inside
// the stream, never decreasing, the last one its length (refused before any
// copy to HBM); that the entries are the stream's element boundaries is
// checked by the decode itself (K4 + sidecar_verdict)
bool index_fits(const uint64_t *idx, size_t count, size_t units, uint64_t clen)
{
    const uint64_t off_mask = (1ull << SNAPPY_AMD_IDX_OFFSET_BITS) - 1;
    if (count != units + 1 || (idx[units] & off_mask) != clen) return false;
    for (size_t i = 0; i < units; i++)
        if ((idx[i] & off_mask) > (idx[i + 1] & off_mask)) return false;
    return true;
}

// A decode driven by a sidecar index failed (rc): it is the index's fault when
// it is not the stream's own block index.  K4 refuses (SNAPPY_AMD_ERR_INDEX) a
// SINGLE unit whose element chain does not end at the next entry, so a decode
// that succeeds had the stream's own index; a failing one is settled here by
// building that index (K5p) and comparing: a different sidecar -> ERR_INDEX,
// the same -> the stream's error, exactly what the decode without a sidecar
// reports (the index pass's own error when the stream cannot be indexed).
int sidecar_verdict(snappy_amd_ctx *c, const uint8_t *d_stream, size_t n, const uint64_t *idx, size_t count, int rc)
{
    if (rc == SNAPPY_AMD_OK || rc == SNAPPY_AMD_ERR_DEVICE) return rc;
    size_t got = 0;
    int r = snappy_amd_index_device(c, d_stream, n, c->d_idx, count, &got);
    if (r) return r;
    std::vector<uint64_t> own(count);
    HIP_OK(hipMemcpy(own.data(), c->d_idx, count * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return memcmp(own.data(), idx, count * sizeof(uint64_t)) ? SNAPPY_AMD_ERR_INDEX : rc;
}

// the largest output a valid stream of n compressed bytes can declare: a
// 3-byte copy-2 element writes at most 64 bytes (src/snappy_decompression.c:
// 290-333), so no stream expands by more than 64/3; a preamble promising more
// is a truncated stream, refused before any output is allocated or mapped
bool length_plausible(uint64_t N, uint64_t n) { return N / 22 <= n; }
}  // namespace

int snappy_amd_host_set_device(int device)
{
    int count = 0;
    if (device >= 0 && (hipGetDeviceCount(&count) != hipSuccess || device >= count)) return SNAPPY_AMD_ERR_DEVICE;
    t_host_device = device < 0 ? -1 : device;
    return SNAPPY_AMD_OK;
}

int snappy_amd_host_get_device(void) { return host_device(); }

int snappy_amd_host_release(void)
{
    std::vector<HostCtx *> idle;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        idle.swap(g_pool);
    }
    for (HostCtx *h : idle) host_free(h);
    return SNAPPY_AMD_OK;
}

size_t snappy_amd_host_pool_size(void)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    return g_pool.size();
}

// A host buffer of more than one 64 MiB chunk: each chunk (a multiple of the
// 65,536-byte block, so the bytes are those of the one-shot stream; chunks
// after the first without the preamble) goes to one of pipe_lanes() contexts of
// its own stream -- H2D, K1r/K3/K2, the compressed size back to pinned memory
// -- so the chunks' copies and kernels overlap and their kernels fill the chip
// together (one 64 MiB chunk is 1,024 blocks on 3,072 wave slots); the
// compressed chunks come back in order, each to the offset its predecessors'
// sizes give.  A lane is reused once its previous chunk has come back.
int host_compress_pipelined(HostCtx &h, const uint8_t *in, size_t n, uint64_t header_value, uint8_t *out,
                            size_t cap, size_t *out_len)
{
    const size_t kPipeChunk = pipe_chunk();
    const size_t nch = (n + kPipeChunk - 1) / kPipeChunk;
    const int lanes = (int)std::min<size_t>((size_t)pipe_lanes(), nch);
    int rc;
    // lane 0 is the host context's own: every stream takes one of the process's
    // hardware queues (GPU_MAX_HW_QUEUES, 4 by default), and a lane that shares
    // one with another stream waits behind that stream's work (a fourth lane of
    // its own queued its K1r behind another lane's K2: profiles/r04e_host_trace_*)
    h.pipe[0] = h.c;
    for (int i = 1; i < lanes; i++)
        if (!h.pipe[i]) {
            if ((rc = create_host_ctx(h.device, &h.pipe[i]))) {
                h.pipe[i] = nullptr;
                return rc;
            }
            high_priority_stream(h.pipe[i]);
        }
    // on an error return, no lane may still be copying from `in` (the caller
    // may free it) or be busy when the context goes back to the pool
    struct LaneGuard {
        HostCtx &h;
        int lanes;
        bool armed = true;
        ~LaneGuard()
        {
            if (armed)
                for (int i = 0; i < lanes; i++)
                    if (h.pipe[i]) (void)hipStreamSynchronize(h.pipe[i]->stream);
        }
    } guard{h, lanes};
    size_t off = 0;  // compressed bytes placed so far
    auto drain = [&](size_t k) -> int {
        snappy_amd_ctx *c = h.pipe[k % (size_t)lanes];
        HIP_OK(hipStreamSynchronize(c->stream));
        const size_t len = (size_t)*c->h_total;
        if (off + len > cap) return SNAPPY_AMD_ERR_CAPACITY;
        HIP_OK(hipMemcpyAsync(out + off, c->d_b, len, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        off += len;
        return SNAPPY_AMD_OK;
    };
    for (size_t k = 0; k < nch; k++) {
        if (k >= (size_t)lanes && (rc = drain(k - (size_t)lanes))) return rc;
        snappy_amd_ctx *c = h.pipe[k % (size_t)lanes];
        const size_t m = std::min(kPipeChunk, n - k * kPipeChunk);
        const size_t units = (m + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
        if ((rc = grow(reinterpret_cast<void **>(&c->d_a), &c->d_a_cap, m + 16)) ||
            (rc = grow(reinterpret_cast<void **>(&c->d_b), &c->d_b_cap,
                       snappy_amd_max_output(m, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE))) ||
            (rc = grow(reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap, (units + 1) * sizeof(uint64_t))))
            return rc;
        HIP_OK(hipMemcpyAsync(c->d_a, in + k * kPipeChunk, m, hipMemcpyHostToDevice, c->stream));
        if ((rc = compress_impl(c, c->d_a, m, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, k ? SNAPPY_AMD_NO_PREAMBLE : 0,
                                header_value, c->d_b, c->d_idx, nullptr)))
            return rc;
        HIP_OK(hipMemcpyAsync(c->h_total, c->total, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    }
    for (size_t k = nch > (size_t)lanes ? nch - (size_t)lanes : 0; k < nch; k++)
        if ((rc = drain(k))) return rc;
    guard.armed = false;  // (every lane drained)
    *out_len = off;
    return SNAPPY_AMD_OK;
}

int snappy_amd_host_compress(const uint8_t *in, size_t n, uint64_t header_value, uint8_t *out, size_t cap,
                             size_t *out_len)
{
    if (!out_len || (!in && n)) return SNAPPY_AMD_ERR_ARG;
    *out_len = 0;
    if (n == 0) return SNAPPY_AMD_OK;
    Lease h(host_device());
    if (h.rc()) return h.rc();
    if (n > pipe_chunk()) return host_compress_pipelined(*h, in, n, header_value, out, cap, out_len);
    size_t len = 0;
    int rc = host_compress_stage(*h, in, n, 0, header_value, &len);
    if (rc) return rc;
    if (len > cap) return SNAPPY_AMD_ERR_CAPACITY;
    HIP_OK(hipMemcpyAsync(out, h->c->d_b, len, hipMemcpyDeviceToHost, h->c->stream));
    HIP_OK(hipStreamSynchronize(h->c->stream));
    *out_len = len;
    return SNAPPY_AMD_OK;
}

int snappy_amd_host_compress_file(FILE *fin, uint64_t header_value, FILE *fout, FILE *fidx, uint64_t *bytes_in)
{
    if (!fin || !fout) return SNAPPY_AMD_ERR_ARG;
    uint64_t base = 0;  // stream bytes written so far
    long idx_hdr = -1;
    if (fidx) {  // sidecar header; N and the entry count are patched at the end
        idx_hdr = ftell(fidx);
        const uint64_t h[3] = {SNAPPY_AMD_IDX_MAGIC, header_value, 0};
        if (idx_hdr < 0 || fwrite(h, sizeof(uint64_t), 3, fidx) != 3) return SNAPPY_AMD_ERR_IO;
    }
    const int dev = host_device();
    Lease hc(dev);
    if (hc.rc()) return hc.rc();
    StreamSlot *slots = hc->slots;
    IoFile in, out;
    AsyncWriter wr;  // (declared after out: joined before out is destroyed)
    if (!in.open(fin, false) || !out.open(fout, true)) return SNAPPY_AMD_ERR_IO;
    // (the output stays on pwrite: mapping it, its fresh pages were allocated by
    // 8 faulting threads, 0.59 -> 0.77 s of writes for 2.3 GB on the GPU box's tmpfs)
    const bool out_mapped = false;
    int rc;
    for (int i = 0; i < 2; i++) {
        StreamSlot &s = slots[i];
        if ((rc = slot_init(s, dev))) return rc;
        if (s.busy) {  // left over by a failed call: discard
            (void)hipStreamSynchronize(s.c->stream);
            s.busy = false;
        }
    }
    HIP_OK(hipSetDevice(dev));
    uint64_t total_in = 0;
    const double t0 = io_now();
    double t_rd = 0, t_dr = 0;
    size_t n = in.read(slots[0].h_in, kStreamChunk);
    t_rd += io_now() - t0;
    if (in.error()) return SNAPPY_AMD_ERR_IO;
    for (uint32_t k = 0; n > 0; k++) {
        StreamSlot &s = slots[k & 1];
        StreamSlot &o = slots[(k + 1) & 1];
        s.n = n;
        total_in += n;
        HIP_OK(hipMemcpyAsync(s.d_in, s.h_in, n, hipMemcpyHostToDevice, s.c->stream));
        rc = compress_impl(s.c, s.d_in, n, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, k ? SNAPPY_AMD_NO_PREAMBLE : 0,
                           header_value, s.d_out, s.d_idx, nullptr);
        if (rc) return rc;
        HIP_OK(hipMemcpyAsync(s.c->h_total, s.c->total, sizeof(uint64_t), hipMemcpyDeviceToHost, s.c->stream));
        s.busy = true;
        // chunk k-1 out while chunk k runs, then chunk k+1 in (its slot is free
        // once chunk k-1 drained)
        const double td = io_now();
        if ((rc = slot_drain(o, wr, out, fidx, &base))) return rc;
        const double tr = io_now();
        n = in.read(o.h_in, kStreamChunk);
        t_rd += io_now() - tr;
        t_dr += tr - td;
        if (in.error()) return SNAPPY_AMD_ERR_IO;
    }
    // the slots drain in chunk order: the one holding the last chunk goes last
    const uint32_t last = total_in ? (uint32_t)(((total_in + kStreamChunk - 1) / kStreamChunk - 1) & 1) : 0;
    if ((rc = slot_drain(slots[last ^ 1], wr, out, fidx, &base))) return rc;
    if ((rc = slot_drain(slots[last], wr, out, fidx, &base))) return rc;
    wr.wait();
    if (!wr.ok) return SNAPPY_AMD_ERR_IO;
    if (!in.finish() || !out.finish()) return SNAPPY_AMD_ERR_IO;
    if (io_trace())
        fprintf(stderr, "[snappy_amd io] compress %llu -> %llu B: %.3f s (reads %.3f, drains %.3f, writes %.3f overlapped), %d/%d threads, "
                        "positional in %d out %d mapped %d\n",
                (unsigned long long)total_in, (unsigned long long)base, io_now() - t0, t_rd, t_dr, wr.busy, io_threads(),
                io_wthreads(), (int)in.pos_io, (int)out.pos_io, (int)out_mapped);
    if (fidx) {
        // the stream's preamble says header_value; an index is only valid for a
        // stream whose preamble is the length actually compressed
        if (total_in != header_value) return SNAPPY_AMD_ERR_INDEX;
        const uint64_t units = (total_in + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
        const uint64_t cnt = total_in ? units + 1 : 0;
        if (total_in && fwrite(&base, sizeof(uint64_t), 1, fidx) != 1) return SNAPPY_AMD_ERR_IO;
        // an index describes the blocks actually written: N = the bytes read
        const uint64_t h[2] = {total_in, cnt};
        if (fseek(fidx, idx_hdr + 8, SEEK_SET) || fwrite(h, sizeof(uint64_t), 2, fidx) != 2 ||
            fseek(fidx, 0, SEEK_END))
            return SNAPPY_AMD_ERR_IO;
    }
    if (bytes_in) *bytes_in = total_in;
    return SNAPPY_AMD_OK;
}

int snappy_amd_host_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len)
{
    return snappy_amd_host_decompress_idx(in, n, nullptr, 0, out, cap, out_len);
}

int snappy_amd_host_decompress_idx(const uint8_t *in, size_t n, const uint64_t *idx, size_t count, uint8_t *out,
                                   size_t cap, size_t *out_len)
{
    if (!out_len || (!in && n)) return SNAPPY_AMD_ERR_ARG;
    *out_len = 0;
    if (n == 0) return SNAPPY_AMD_OK;
    uint64_t N = 0;
    if (snappy_varint_decode(in, n, &N) == 0) return SNAPPY_AMD_ERR_HEADER;
    if (N > cap) return SNAPPY_AMD_ERR_CAPACITY;
    if (!length_plausible(N, n)) return SNAPPY_AMD_ERR_TRUNCATED;
    Lease h(host_device());
    if (h.rc()) return h.rc();
    snappy_amd_ctx *c = h->c;
    const size_t units = (N + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    int rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_a), &c->d_a_cap, n + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_b), &c->d_b_cap, N + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap, (units + 2) * sizeof(uint64_t)))) return rc;
    HIP_OK(hipMemcpyAsync(c->d_a, in, n, hipMemcpyHostToDevice, c->stream));
    if (idx) {  // a sidecar index: no index pass; it must describe this stream
        if (!index_fits(idx, count, units, n)) return SNAPPY_AMD_ERR_INDEX;
        HIP_OK(hipMemcpyAsync(c->d_idx, idx, count * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    } else {
        size_t got = 0;
        rc = snappy_amd_index_device(c, c->d_a, n, c->d_idx, units + 1, &got);
        if (rc) return rc;
    }
    if (N == 0) { *out_len = 0; return SNAPPY_AMD_OK; }
    rc = snappy_amd_decompress_device(c, c->d_a, c->d_idx, (size_t)N, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, c->d_b);
    if (rc && idx) rc = sidecar_verdict(c, c->d_a, n, idx, count, rc);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, c->d_b, N, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    *out_len = (size_t)N;
    return SNAPPY_AMD_OK;
}

int snappy_amd_host_decompress_file(FILE *fin, const uint64_t *idx, size_t count, FILE *fout)
{
    if (!fin || !fout) return SNAPPY_AMD_ERR_ARG;
    IoFile in, out;
    if (!in.open(fin, false) || !in.pos_io) return SNAPPY_AMD_ERR_UNSUPPORTED;
    const uint64_t n = in.remaining();
    if (n == 0) return in.finish() ? SNAPPY_AMD_OK : SNAPPY_AMD_ERR_IO;  // nothing to decode, nothing written
    Lease h(host_device());
    if (h.rc()) return h.rc();
    snappy_amd_ctx *c = h->c;
    DecStage &dec = h->dec;
    int rc;
    if ((rc = dec_stage_init(dec))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_a), &c->d_a_cap, n + 16))) return rc;
    // the output's pages are allocated (file size unchanged) from the moment
    // the header gives N, while the input is read and the index and decode
    // run: the writes then only copy (GPU box tmpfs: 10.5 GB/s against 5.8
    // into fresh pages; one file's allocation and writes serialise on its
    // inode, so this is the overlap there is).  Best effort: a file system
    // without fallocate just skips it.
    if (!out.open(fout, true)) return SNAPPY_AMD_ERR_IO;
    // On any failure after the preallocation started, the blocks it added past
    // the file's old end and past what was written are released (they are
    // invisible in the file size); the thread is joined first.  Declared after
    // `out`, so this runs before out's unmap / truncation.
    struct Prealloc {
        IoFile &out;
        std::thread t;
        uint64_t at = 0, len = 0, old_size = 0;
        bool ok = false;
        ~Prealloc()
        {
            if (t.joinable()) t.join();
            if (ok || !len) return;
            const uint64_t from = std::max(std::max(at, old_size), out.pos), end = at + len;
            if (end > from)
                (void)fallocate(out.fd, FALLOC_FL_PUNCH_HOLE | FALLOC_FL_KEEP_SIZE, (off_t)from, (off_t)(end - from));
        }
    } pre{out};
    // (1) file -> pinned chunk k % 3 (host threads) -> HBM (copy engine), the
    // next chunk read while this one is copied
    const double t0 = io_now();
    double t_rd = 0;
    uint64_t N = 0;
    bool out_mapped = false;
    const uint64_t nch = (n + kStreamChunk - 1) / kStreamChunk;
    for (uint64_t k = 0; k < nch; k++) {
        const int s = (int)(k % 3);
        if (k >= 3) HIP_OK(hipEventSynchronize(dec.ev[s]));
        const size_t m = (size_t)std::min<uint64_t>(kStreamChunk, n - k * kStreamChunk);
        const double tr = io_now();
        if (in.read(dec.h[s], m) != m) return SNAPPY_AMD_ERR_IO;
        t_rd += io_now() - tr;
        if (k == 0) {
            if (snappy_varint_decode(dec.h[0], m, &N) == 0) return SNAPPY_AMD_ERR_HEADER;
            // N is untrusted until the decode succeeds: bounded by what n bytes
            // can expand to before the output is mapped or preallocated
            if (!length_plausible(N, n)) return SNAPPY_AMD_ERR_TRUNCATED;
            if (out.pos_io && N) {
                struct stat st;
                pre.old_size = fstat(out.fd, &st) == 0 ? (uint64_t)st.st_size : 0;
                pre.at = out.pos;
                pre.len = N;
                // map first: its ftruncate would wait for the whole fallocate (both take the inode lock)
                out_mapped = out.map_out(N);
                pre.t = std::thread([fd = out.fd, at = out.pos, N] {
                    (void)fallocate(fd, FALLOC_FL_KEEP_SIZE, (off_t)at, (off_t)N);
                });
            }
        }
        HIP_OK(hipMemcpyAsync(c->d_a + k * kStreamChunk, dec.h[s], m, hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipEventRecord(dec.ev[s], c->stream));
    }
    if (!in.finish()) return SNAPPY_AMD_ERR_IO;
    const double t1 = io_now();
    // (2) block index (sidecar, checked, or the GPU index pass) and decode
    const uint64_t units = (N + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_b), &c->d_b_cap, N + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap, (units + 2) * sizeof(uint64_t)))) return rc;
    if (idx) {
        if (!index_fits(idx, count, units, n)) return SNAPPY_AMD_ERR_INDEX;
        HIP_OK(hipMemcpyAsync(c->d_idx, idx, count * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    } else {
        size_t got = 0;
        if ((rc = snappy_amd_index_device(c, c->d_a, n, c->d_idx, units + 1, &got))) return rc;
    }
    if (N == 0) {
        pre.ok = true;
        return SNAPPY_AMD_OK;
    }
    rc = snappy_amd_decompress_device(c, c->d_a, c->d_idx, (size_t)N, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, c->d_b);
    if (rc && idx) rc = sidecar_verdict(c, c->d_a, n, idx, count, rc);
    if (rc) return rc;
    // (3) HBM -> pinned chunk (copy engine) -> file (a writer thread, itself
    // using several threads on a mapped output)
    const double t2 = io_now();
    double t_wr = 0;
    // the mapped writers need not wait for the preallocation: a page it has not
    // reached yet is allocated by the writer's populate (the preallocation skips it)
    if (!out_mapped && pre.t.joinable()) pre.t.join();
    const double t3 = io_now();
    const uint64_t och = (N + kStreamChunk - 1) / kStreamChunk;
    auto down = [&](uint64_t k) -> int {
        const size_t m = (size_t)std::min<uint64_t>(kStreamChunk, N - k * kStreamChunk);
        HIP_OK(hipMemcpyAsync(dec.h[k % 3], c->d_b + k * kStreamChunk, m, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipEventRecord(dec.ev[k % 3], c->stream));
        return SNAPPY_AMD_OK;
    };
    // two chunks copied down ahead of the one being written (by the writer thread:
    // chunk k's slot is refilled with chunk k + 3 once its write has been joined)
    if ((rc = down(0))) return rc;
    if (och > 1 && (rc = down(1))) return rc;
    AsyncWriter wr;  // (after out and pre: joined before either is destroyed)
    double t_ev = 0, t_join = 0;
    for (uint64_t k = 0; k < och; k++) {
        const double te = io_now();
        HIP_OK(hipEventSynchronize(dec.ev[k % 3]));
        const size_t m = (size_t)std::min<uint64_t>(kStreamChunk, N - k * kStreamChunk);
        const double tj = io_now();
        t_ev += tj - te;
        const bool started = wr.start(out, dec.h[k % 3], m);  // joins chunk k - 1's write
        t_join += io_now() - tj;
        if (!started) return SNAPPY_AMD_ERR_IO;
        if (k + 2 < och && (rc = down(k + 2))) return rc;                 // into chunk k - 1's slot
    }
    wr.wait();
    t_wr = wr.busy;
    if (!wr.ok) return SNAPPY_AMD_ERR_IO;
    const double t4 = io_now();
    const bool fin_ok = out.finish();
    pre.ok = fin_ok;
    if (io_trace())
        fprintf(stderr, "[snappy_amd io] decompress %llu -> %llu B: in %.3f s (reads %.3f), index+decode %.3f s, "
                        "preallocation wait %.3f s, out %.3f s (copy waits %.3f, writer waits %.3f, writes %.3f, "
                        "finish %.3f), %d/%d threads, positional out %d mapped %d\n",
                (unsigned long long)n, (unsigned long long)N, t1 - t0, t_rd, t2 - t1, t3 - t2, io_now() - t3, t_ev,
                t_join, t_wr, io_now() - t4,
                io_threads(), io_wthreads(), (int)out.pos_io, (int)out_mapped);
    return fin_ok ? SNAPPY_AMD_OK : SNAPPY_AMD_ERR_IO;
}

// ---- several devices from one host call (SURVEY 8(e) for C callers) -------
//
// The host-buffer API over a list of devices: the 65,536-byte blocks of the
// input are split into contiguous ranges, one per device (rounded up as
// dist.shard_range: the first device holds the first block and writes the
// preamble, the others compress with SNAPPY_AMD_NO_PREAMBLE), each compressed
// on its device by its own thread and host context; once every size is known
// (the C1 step) each device copies its bytes to their final offset in `out`
// (the C2 step: the gather is the host buffer).  The output is byte-identical
// to snappy_compress_buffer's.  A device may appear more than once (two
// contexts on one device, as the tests do on a 1-GPU box).
}  // extern "C"

namespace {
struct Shard {
    size_t u0 = 0, u1 = 0;
};
std::vector<Shard> split_units(size_t units, int parts)
{
    std::vector<Shard> s((size_t)parts);
    for (int r = 0; r < parts; r++) {
        s[(size_t)r].u0 = (units * (size_t)r + (size_t)parts - 1) / (size_t)parts;
        s[(size_t)r].u1 = (units * (size_t)(r + 1) + (size_t)parts - 1) / (size_t)parts;
    }
    return s;
}

template <class F>
void on_threads(int parts, F f)
{
    std::vector<std::thread> th;
    for (int r = 1; r < parts; r++) th.emplace_back(f, r);
    f(0);
    for (auto &t : th) t.join();
}
}  // namespace

extern "C" {

int snappy_compress_buffer_multi(const int *devices, int ndev, const uint8_t *in, size_t n, uint8_t *out,
                                 size_t *out_len)
{
    if (!out_len || !devices || ndev < 1 || (n && (!in || !out))) return SNAPPY_AMD_ERR_ARG;
    *out_len = 0;
    if (n == 0) return SNAPPY_AMD_OK;
    const size_t units = (n + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    const int parts = (int)std::min<size_t>((size_t)ndev, units);
    const std::vector<Shard> sh = split_units(units, parts);
    std::vector<std::unique_ptr<Lease>> lease((size_t)parts);
    for (int r = 0; r < parts; r++) {
        lease[(size_t)r].reset(new Lease(devices[r]));
        if (lease[(size_t)r]->rc()) return lease[(size_t)r]->rc();
    }
    std::vector<size_t> len((size_t)parts, 0);
    std::vector<int> rc((size_t)parts, SNAPPY_AMD_OK);
    on_threads(parts, [&](int r) {  // compress every range on its device
        const size_t off = sh[(size_t)r].u0 * SNAPPY_AMD_BLOCK;
        const size_t m = std::min(n, sh[(size_t)r].u1 * SNAPPY_AMD_BLOCK) - off;
        HostCtx &h = **lease[(size_t)r];
        if (hipSetDevice(h.device) != hipSuccess) { rc[(size_t)r] = SNAPPY_AMD_ERR_DEVICE; return; }
        rc[(size_t)r] = host_compress_stage(h, in + off, m, r ? SNAPPY_AMD_NO_PREAMBLE : 0, (uint64_t)n,
                                            &len[(size_t)r]);
    });
    for (int r = 0; r < parts; r++)
        if (rc[(size_t)r]) return rc[(size_t)r];
    std::vector<size_t> at((size_t)parts + 1, 0);  // C1: each range's offset in the stream
    for (int r = 0; r < parts; r++) at[(size_t)r + 1] = at[(size_t)r] + len[(size_t)r];
    if (at[(size_t)parts] > snappy_max_compressed_length(n)) return SNAPPY_AMD_ERR_CAPACITY;
    on_threads(parts, [&](int r) {  // C2: every range to its place in out
        HostCtx &h = **lease[(size_t)r];
        if (hipSetDevice(h.device) != hipSuccess ||
            hipMemcpyAsync(out + at[(size_t)r], h.c->d_b, len[(size_t)r], hipMemcpyDeviceToHost, h.c->stream) !=
                hipSuccess ||
            hipStreamSynchronize(h.c->stream) != hipSuccess)
            rc[(size_t)r] = SNAPPY_AMD_ERR_DEVICE;
    });
    for (int r = 0; r < parts; r++)
        if (rc[(size_t)r]) return rc[(size_t)r];
    *out_len = at[(size_t)parts];
    return SNAPPY_AMD_OK;
}

// Decoding over several devices: the first device copies the whole stream in
// and builds its block index (K5p); each device then decodes a contiguous
// block range from its part of the stream.  A range must start on an element
// boundary and may not copy from an earlier range (streams this library
// writes never do: their blocks are self-contained); otherwise -- elements
// straddling a range start, or a range reporting SNAPPY_AMD_ERR_OFFSET -- the
// first device decodes the whole stream, so every stream snappy_decompress
// accepts is accepted here, with the same result.
int snappy_decompress_buffer_multi(const int *devices, int ndev, const uint8_t *in, size_t n, uint8_t *out, size_t cap,
                                   size_t *out_len)
{
    if (!out_len || !devices || ndev < 1 || (n && !in)) return SNAPPY_AMD_ERR_ARG;
    *out_len = 0;
    if (n == 0) return SNAPPY_AMD_OK;
    uint64_t N = 0;
    if (snappy_varint_decode(in, n, &N) == 0) return SNAPPY_AMD_ERR_HEADER;
    if (N > cap) return SNAPPY_AMD_ERR_CAPACITY;
    if (N && !out) return SNAPPY_AMD_ERR_ARG;
    if (!length_plausible(N, n)) return SNAPPY_AMD_ERR_TRUNCATED;
    const size_t units = (N + SNAPPY_AMD_BLOCK - 1) / SNAPPY_AMD_BLOCK;
    const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)ndev, units));
    std::vector<std::unique_ptr<Lease>> lease((size_t)parts);
    for (int r = 0; r < parts; r++) {
        lease[(size_t)r].reset(new Lease(devices[r]));
        if (lease[(size_t)r]->rc()) return lease[(size_t)r]->rc();
    }
    snappy_amd_ctx *c0 = (*lease[0])->c;
    int rc;
    if ((rc = grow(reinterpret_cast<void **>(&c0->d_a), &c0->d_a_cap, n + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c0->d_b), &c0->d_b_cap, N + 16))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c0->d_idx), &c0->d_idx_cap, (units + 2) * sizeof(uint64_t)))) return rc;
    HIP_OK(hipSetDevice(c0->device));
    HIP_OK(hipMemcpyAsync(c0->d_a, in, n, hipMemcpyHostToDevice, c0->stream));
    size_t got = 0;
    if ((rc = snappy_amd_index_device(c0, c0->d_a, n, c0->d_idx, units + 1, &got))) return rc;
    if (N == 0) return SNAPPY_AMD_OK;
    std::vector<uint64_t> idx(units + 1);
    HIP_OK(hipMemcpy(idx.data(), c0->d_idx, (units + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    const std::vector<Shard> sh = split_units(units, parts);
    const uint64_t off_mask = (1ull << SNAPPY_AMD_IDX_OFFSET_BITS) - 1;
    bool split = parts > 1;
    for (int r = 1; r < parts && split; r++) split = (idx[sh[(size_t)r].u0] >> SNAPPY_AMD_IDX_OFFSET_BITS) == 0;
    std::vector<int> rcs((size_t)parts, SNAPPY_AMD_OK);
    if (split) {
        on_threads(parts, [&](int r) {
            HostCtx &h = **lease[(size_t)r];
            snappy_amd_ctx *c = h.c;
            const size_t u0 = sh[(size_t)r].u0, u1 = sh[(size_t)r].u1;
            const size_t o0 = u0 * SNAPPY_AMD_BLOCK, m = std::min<uint64_t>(N, u1 * SNAPPY_AMD_BLOCK) - o0;
            int e = SNAPPY_AMD_OK;
            if (hipSetDevice(h.device) != hipSuccess) e = SNAPPY_AMD_ERR_DEVICE;
            if (!e && r == 0) {  // the first range decodes in place from the whole stream
                e = snappy_amd_decompress_device_ex(c, c->d_a, c->d_idx, m, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE, 0,
                                                    N, c->d_b, 1);
            } else if (!e) {
                const uint64_t b0 = idx[u0] & off_mask, b1 = idx[u1] & off_mask;
                std::vector<uint64_t> loc(u1 - u0 + 1);
                for (size_t u = u0; u <= u1; u++) loc[u - u0] = (idx[u] & off_mask) - b0 + (idx[u] & ~off_mask);
                if ((e = grow(reinterpret_cast<void **>(&c->d_a), &c->d_a_cap, (size_t)(b1 - b0) + 16)) ||
                    (e = grow(reinterpret_cast<void **>(&c->d_b), &c->d_b_cap, m + 16)) ||
                    (e = grow(reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap, loc.size() * sizeof(uint64_t)))) {
                } else if (hipMemcpyAsync(c->d_a, in + b0, (size_t)(b1 - b0), hipMemcpyHostToDevice, c->stream) !=
                               hipSuccess ||
                           hipMemcpyAsync(c->d_idx, loc.data(), loc.size() * sizeof(uint64_t), hipMemcpyHostToDevice,
                                          c->stream) != hipSuccess) {
                    e = SNAPPY_AMD_ERR_DEVICE;
                } else {
                    e = snappy_amd_decompress_device_ex(c, c->d_a, c->d_idx, m, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE,
                                                        SNAPPY_AMD_NO_PREAMBLE, N, c->d_b, 1);
                }
            }
            if (!e && (hipMemcpyAsync(out + o0, c->d_b, m, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                       hipStreamSynchronize(c->stream) != hipSuccess))
                e = SNAPPY_AMD_ERR_DEVICE;
            rcs[(size_t)r] = e;
        });
        // the first failing range in order decides, as the first failing unit
        // does for one device: ERR_OFFSET from a range after the first may be a
        // legal copy from an earlier range, so the whole stream is decoded on
        // one device (which then reports whatever error comes first)
        bool again = false;
        for (int r = 0; r < parts && !again; r++) {
            if (rcs[(size_t)r] == SNAPPY_AMD_ERR_OFFSET && r > 0) again = true;
            else if (rcs[(size_t)r]) return rcs[(size_t)r];
        }
        if (!again) {
            *out_len = (size_t)N;
            return SNAPPY_AMD_OK;
        }
    }
    // one device decodes the whole stream (ordered second pass for cross-block copies)
    HIP_OK(hipSetDevice(c0->device));
    if ((rc = snappy_amd_decompress_device(c0, c0->d_a, c0->d_idx, (size_t)N, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE,
                                           c0->d_b)))
        return rc;
    HIP_OK(hipMemcpyAsync(out, c0->d_b, N, hipMemcpyDeviceToHost, c0->stream));
    HIP_OK(hipStreamSynchronize(c0->stream));
    *out_len = (size_t)N;
    return SNAPPY_AMD_OK;
}

}  // extern "C"
