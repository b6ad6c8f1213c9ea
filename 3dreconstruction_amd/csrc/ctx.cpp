// Context management, error reporting and the run-time RCCL binding.
#include <dlfcn.h>
#include <malloc.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

#include "common.h"

namespace sfm {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl* rccl() {
    static Rccl r;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.all_gather &&
             r.error_string;
    });
    SFM_REQUIRE(ok, SFM_ERR_COMM, "RCCL (librccl.so.1) not available");
    return &r;
}

int rccl_comm_init(void** comm, int world, const uint8_t* id128, int rank) {
    const Rccl* r = rccl();
    ncclUniqueId id;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(&id, id128, 128);
    ncclComm_t c = nullptr;
    ncclResult_t e = r->comm_init_rank(&c, world, id, rank);
    SFM_REQUIRE(e == ncclSuccess, SFM_ERR_COMM, "ncclCommInitRank: %s", r->error_string(e));
    *comm = c;
    return SFM_OK;
}

void rccl_comm_destroy(void* comm) {
    if (comm) rccl()->comm_destroy((ncclComm_t)comm);
}

int rccl_allreduce_f64(void* comm, double* buf, size_t n, int op_max, hipStream_t s) {
    const Rccl* r = rccl();
    ncclResult_t e = r->all_reduce(buf, buf, n, ncclFloat64, op_max ? ncclMax : ncclSum,
                                   (ncclComm_t)comm, s);
    SFM_REQUIRE(e == ncclSuccess, SFM_ERR_COMM, "ncclAllReduce: %s", r->error_string(e));
    return SFM_OK;
}

int rccl_allgather_f64(void* comm, const double* in, double* out, size_t n, hipStream_t s) {
    const Rccl* r = rccl();
    ncclResult_t e = r->all_gather(in, out, n, ncclFloat64, (ncclComm_t)comm, s);
    SFM_REQUIRE(e == ncclSuccess, SFM_ERR_COMM, "ncclAllGather: %s", r->error_string(e));
    return SFM_OK;
}

void set_dyn_lds(const void* kernel, size_t bytes) {
    int dev = 0;
    SFM_HIP(hipGetDevice(&dev));
    // hot path: a thread that has already seen the attribute raised
    // far enough for this (device, kernel) returns without the process-wide
    // lock -- the BCR / dense solves call this several times per LM iteration
    struct Seen {
        int dev;
        const void* kernel;
        size_t bytes;
    };
    thread_local std::vector<Seen> seen;
    for (const Seen& x : seen)
        if (x.dev == dev && x.kernel == kernel && x.bytes >= bytes) return;
    static std::mutex mu;
    static auto* done = new std::map<std::pair<int, const void*>, size_t>;   // never destroyed
    std::lock_guard<std::mutex> lk(mu);
    size_t& have = (*done)[{dev, kernel}];
    if (have < bytes) {
        SFM_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        have = bytes;
    }
    for (Seen& x : seen)
        if (x.dev == dev && x.kernel == kernel) {
            x.bytes = have;
            return;
        }
    seen.push_back({dev, kernel, have});
}

int device_cu_count() {
    int dev = 0;
    SFM_HIP(hipGetDevice(&dev));
    static std::mutex mu;
    static auto* cus = new std::map<int, int>;
    std::lock_guard<std::mutex> lk(mu);
    int& n = (*cus)[dev];
    if (!n) SFM_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return n;
}

// ---- device memory cache ----------------------------------------------------
namespace {

thread_local hipStream_t tl_stream = nullptr;   // key of the bound context

// Size classes: 256 B granules up to 64 KB, above that eight classes per
// power of two (<= 12.5 % slack), so regrown buffers of a growing problem
// (the incremental loop) still find their class.
size_t size_class(size_t b) {
    if (b <= 65536) return (b + 255) & ~size_t(255);
    int e = 63 - __builtin_clzll(b - 1);          // 2^e < b <= 2^(e+1)
    const size_t step = size_t(1) << (e - 2);     // 2^(e+1) / 8
    return (b + step - 1) / step * step;
}

// kind 0: device, 1: pinned mapped + coherent (polled scalars), 2: pinned
// staging for uploads
struct Block {
    hipStream_t key;
    size_t bytes;
    int kind;
};

struct MemCache {
    std::mutex mu;
    std::unordered_map<void*, Block> live;
    // (key, kind, class) -> free blocks
    std::map<std::tuple<hipStream_t, int, size_t>, std::vector<void*>> free;
    std::unordered_set<hipStream_t> streams;   // contexts alive (their keys)
    size_t cached = 0;
    static constexpr size_t kCap = size_t(32) << 30;   // cached bytes kept at most
};

MemCache& cache() {
    static MemCache* c = new MemCache;   // never destroyed: frees may run at exit
    return *c;
}

void raw_free(void* p, int kind) {
    if (kind) (void)hipHostFree(p);
    else (void)hipFree(p);
}

void release_all_locked(MemCache& c, hipStream_t only, bool all) {
    for (auto it = c.free.begin(); it != c.free.end();) {
        if (all || std::get<0>(it->first) == only) {
            for (void* p : it->second) {
                raw_free(p, std::get<1>(it->first));
                c.cached -= std::get<2>(it->first);
            }
            it = c.free.erase(it);
        } else {
            ++it;
        }
    }
}

void* cached_alloc(size_t bytes, int kind) {
    MemCache& c = cache();
    const hipStream_t key = tl_stream;
    const size_t cls = size_class(bytes);
    std::lock_guard<std::mutex> lk(c.mu);
    if (key && c.streams.count(key)) {
        auto it = c.free.find({key, kind, cls});
        if (it != c.free.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            c.cached -= cls;
            c.live[p] = Block{key, cls, kind};
            return p;
        }
    }
    void* p = nullptr;
    auto get = [&] {
        return kind == 1   ? hipHostMalloc(&p, cls, hipHostMallocMapped | hipHostMallocCoherent)
               : kind == 2 ? hipHostMalloc(&p, cls, hipHostMallocDefault)
                           : hipMalloc(&p, cls);
    };
    hipError_t e = get();
    if (e != hipSuccess && c.cached) {   // give the cache back and retry once
        (void)hipGetLastError();
        release_all_locked(c, nullptr, true);
        e = get();
    }
    if (e != hipSuccess) {
        set_error("%s(%zu bytes) failed: %s", kind ? "hipHostMalloc" : "hipMalloc", cls, hipGetErrorString(e));
        throw SfmError{SFM_ERR_OOM};
    }
    c.live[p] = Block{key, cls, kind};
    return p;
}

// false when p is not a block of the cache
bool cached_free(void* p) {
    if (!p) return true;
    MemCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return false;
    const Block b = it->second;
    c.live.erase(it);
    // reuse only under the stream the block was allocated and used on: a block
    // freed while another context is bound may still have work queued on its
    // own stream, which the other stream's order does not cover
    const hipStream_t key = b.key;
    if (key && c.streams.count(key) && c.cached + b.bytes <= MemCache::kCap) {
        c.free[{key, b.kind, b.bytes}].push_back(p);
        c.cached += b.bytes;
        return true;
    }
    raw_free(p, b.kind);
    return true;
}

}  // namespace

void* dev_alloc(size_t bytes) { return cached_alloc(bytes, 0); }
void dev_free(void* p) { (void)cached_free(p); }
void* pinned_alloc(size_t bytes) { return cached_alloc(bytes, 1); }
void pinned_free(void* p) { (void)cached_free(p); }
void* host_alloc(size_t bytes) {
    if (tl_stream) return cached_alloc(bytes, 2);
    void* p = std::malloc(std::max<size_t>(bytes, 1));
    if (!p) throw std::bad_alloc();
    return p;
}
void host_free(void* p) {
    if (!cached_free(p)) std::free(p);
}

void dev_cache_release(hipStream_t s) {
    MemCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    release_all_locked(c, s, false);
    c.streams.erase(s);
}

CtxScope::CtxScope(const sfm_ctx* ctx) : prev(tl_stream) {
    SFM_HIP(hipSetDevice(ctx->device));
    tl_stream = ctx->stream;
}
CtxScope::~CtxScope() { tl_stream = prev; }

}  // namespace sfm

using namespace sfm;

extern "C" const char* sfm_version(void) { return "sfmcore 0.1.0 (gfx950)"; }

extern "C" const char* sfm_last_error(void) { return g_err.c_str(); }

void sfm::ctx_allreduce(sfm_ctx* ctx, double* dev_buf, size_t n, int op_max, hipStream_t s) {
    if (n == 0 || (ctx->world <= 1 && !ctx->comm) || ctx->no_exchange) return;   // a 1-rank RCCL comm still runs
    if (!ctx->host_allreduce) {
        SFM_REQUIRE(rccl_allreduce_f64(ctx->comm, dev_buf, n, op_max, s) == 0, SFM_ERR_COMM,
                    "RCCL all-reduce failed");
        return;
    }
    if (ctx->host_cap < n) {
        if (ctx->host_buf) SFM_HIP(hipHostFree(ctx->host_buf));
        ctx->host_buf = nullptr;
        SFM_HIP(hipHostMalloc(&ctx->host_buf, n * sizeof(double)));
        ctx->host_cap = n;
    }
    SFM_HIP(hipMemcpyAsync(ctx->host_buf, dev_buf, n * sizeof(double), hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    SFM_REQUIRE(ctx->host_allreduce(ctx->host_allreduce_user, ctx->host_buf, (int64_t)n, op_max) == 0,
                SFM_ERR_COMM, "host all-reduce hook failed");
    SFM_HIP(hipMemcpyAsync(dev_buf, ctx->host_buf, n * sizeof(double), hipMemcpyHostToDevice, s));
    SFM_HIP(hipStreamSynchronize(s));   // the staging buffer is reused by the next exchange
}

extern "C" int sfm_comm_unique_id(uint8_t* out128) {
    return guarded([&] {
        SFM_REQUIRE(out128, SFM_ERR_INVALID_ARG, "null output");
        ncclUniqueId id;
        ncclResult_t e = rccl()->get_unique_id(&id);
        SFM_REQUIRE(e == ncclSuccess, SFM_ERR_COMM, "ncclGetUniqueId: %s",
                    rccl()->error_string(e));
        std::memcpy(out128, &id, 128);
        return SFM_OK;
    });
}

namespace {
// Unmapping a large host allocation makes the GPU driver invalidate the
// process's device-visible mappings, and the next GPU operation of the process
// waits for it: 12-27 ms after a bundle adjustment freed its ~100 MB of
// planner arrays, which the C5 loop paid before every image's match
// (tools/match_latency.py).  glibc serves allocations above its mmap
// threshold with mmap / munmap; the threshold at its maximum (32 MiB on
// 64-bit: glibc rejects anything above HEAP_MAX_SIZE / 2) and a large trim
// threshold keep freed blocks in the heap for reuse instead.  Opt-in
// (SFM_CTX_TUNE_HOST_MALLOC), once per process: a
// long-running host application keeps its own malloc settings by default.
void tune_host_malloc() {
    static std::once_flag once;
    std::call_once(once, [] {
        const int a = mallopt(M_MMAP_THRESHOLD, 32 << 20);
        const int b = mallopt(M_TRIM_THRESHOLD, 1 << 30);
        if (!a || !b) std::fprintf(stderr, "[sfmcore] mallopt rejected (mmap threshold %d, trim threshold %d)\n", a, b);
    });
}
}  // namespace

extern "C" int sfm_ctx_create(const sfm_ctx_opts* opts, sfm_ctx** out) {
    return guarded([&] {
        SFM_REQUIRE(opts && out, SFM_ERR_INVALID_ARG, "null argument");
        SFM_REQUIRE(opts->world_size >= 1 && opts->rank >= 0 && opts->rank < opts->world_size,
                    SFM_ERR_INVALID_ARG, "bad rank %d / world_size %d", opts->rank,
                    opts->world_size);
        SFM_REQUIRE(((opts->flags >> 12) & 7) <= 4 && ((opts->flags >> 15) & 7) <= 3, SFM_ERR_INVALID_ARG,
                    "bad SFM_CTX_BA_STEP_LANES / SFM_CTX_BA_REDUCE_WAVES field");
        int ndev = 0;
        hipError_t e = hipGetDeviceCount(&ndev);
        SFM_REQUIRE(e == hipSuccess && ndev > 0, SFM_ERR_DEVICE, "no HIP device available (%s)",
                    hipGetErrorString(e));
        SFM_REQUIRE(opts->device >= 0 && opts->device < ndev, SFM_ERR_INVALID_ARG,
                    "device %d out of range (%d devices)", opts->device, ndev);
        hipDeviceProp_t prop;
        SFM_HIP(hipGetDeviceProperties(&prop, opts->device));
        SFM_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, SFM_ERR_DEVICE,
                    "device %d is %s; this build targets gfx950 (MI355X) only", opts->device,
                    prop.gcnArchName);
        if (opts->flags & SFM_CTX_TUNE_HOST_MALLOC) tune_host_malloc();
        auto* c = new sfm_ctx;
        c->device = opts->device;
        c->rank = opts->rank;
        c->world = opts->world_size;
        c->cu_count = prop.multiProcessorCount;
        c->fail_solve_wait = (opts->flags & SFM_CTX_DIAG_FAIL_SOLVE_WAIT) != 0;
        c->time_kernels = (opts->flags & SFM_CTX_TIME_KERNELS) != 0;
        c->flags = opts->flags;
        SFM_HIP(hipSetDevice(c->device));
        SFM_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        {
            MemCache& mc = cache();
            std::lock_guard<std::mutex> lk(mc.mu);
            mc.streams.insert(c->stream);
        }
        if (opts->flags & SFM_CTX_DIAG_NO_EXCHANGE) {
            SFM_REQUIRE(!opts->comm_id && !opts->allreduce, SFM_ERR_INVALID_ARG,
                        "SFM_CTX_DIAG_NO_EXCHANGE excludes a communicator or an all-reduce hook");
            c->no_exchange = true;
        } else if (c->world > 1 && opts->allreduce && !opts->comm_id) {
            c->host_allreduce = opts->allreduce;
            c->host_allreduce_user = opts->allreduce_user;
        } else if (c->world > 1 || opts->comm_id) {   // comm_id at world_size 1: a 1-rank RCCL comm
            SFM_REQUIRE(opts->comm_id, SFM_ERR_INVALID_ARG, "world_size>1 needs comm_id or an allreduce hook");
            try {
                rccl_comm_init(&c->comm, c->world, opts->comm_id, c->rank);
            } catch (...) {
                (void)hipStreamDestroy(c->stream);
                delete c;
                throw;
            }
        }
        *out = c;
        return SFM_OK;
    });
}

extern "C" int sfm_ctx_last_kernel_ms(sfm_ctx* ctx, double* ms) {
    return guarded([&] {
        SFM_REQUIRE(ctx && ms, SFM_ERR_INVALID_ARG, "sfm_ctx_last_kernel_ms: bad arguments");
        *ms = ctx->last_kernel_ms;
        return SFM_OK;
    });
}

extern "C" int sfm_ctx_destroy(sfm_ctx* ctx) {
    return guarded([&] {
        if (!ctx) return SFM_OK;
        (void)hipSetDevice(ctx->device);
        ba_cache_release(ctx);
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        rccl_comm_destroy(ctx->comm);
        if (ctx->host_buf) (void)hipHostFree(ctx->host_buf);
        for (hipEvent_t e : ctx->ev)
            if (e) (void)hipEventDestroy(e);
        if (ctx->stream) {
            dev_cache_release(ctx->stream);
            (void)hipStreamDestroy(ctx->stream);
        }
        delete ctx;
        return SFM_OK;
    });
}

extern "C" int sfm_ctx_synchronize(sfm_ctx* ctx) {
    return guarded([&] {
        SFM_REQUIRE(ctx, SFM_ERR_INVALID_ARG, "null ctx");
        CtxScope scope(ctx);
        SFM_HIP(hipStreamSynchronize(ctx->stream));
        return SFM_OK;
    });
}
