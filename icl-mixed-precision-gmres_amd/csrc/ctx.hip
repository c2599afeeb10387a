// Context, memory and error plumbing of the C-ABI (include/mpgmres/capi.h).
// Replaces the Kokkos::View allocation / deep_copy layer (types.hpp:15-228)
// and the global cuBLAS/cuSPARSE singleton (types_cuda.hpp:9-36): one
// explicit context per (GPU, host thread), no global mutable state.
#include "internal.hpp"

#include <cstdlib>
#include <cstring>
#include <new>

namespace {
// Small device -> host reads (the operator surface's per-cycle residual log):
// one workgroup stores the words straight into the context's pinned staging
// block with system-scope stores, as the host-value reductions do, so a read
// is one kernel on the stream and a polled wait instead of a runtime copy
// (a blit dispatch with a gap of its own before it). MPG_D2H_KERNEL=0: the
// runtime copy.
// With a flag (mpg::host_poll): every lane's stores waited for, then one
// lane stores the sequence number.
__global__ __launch_bounds__(256) void k_d2h_words(const uint32_t* __restrict__ src, uint32_t* dst, int words,
                                                   unsigned* flag, unsigned seq) {
    for (int t = threadIdx.x; t < words; t += blockDim.x)
        __hip_atomic_store(dst + t, src[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!flag) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
bool d2h_kernel() {
    const char* e = std::getenv("MPG_D2H_KERNEL");
    return !(e && *e == '0');
}
}  // namespace

extern "C" {

const char* mpg_error_string(int status) {
    switch (status) {
        case MPG_OK: return "ok";
        case MPG_ERR_HIP: return "HIP runtime error";
        case MPG_ERR_ARG: return "invalid argument";
        case MPG_ERR_ALLOC: return "device allocation failed";
        case MPG_ERR_RCCL: return "RCCL error";
        case MPG_ERR_UNSUPPORTED: return "unsupported operation";
        case MPG_ERR_BREAKDOWN: return "Arnoldi breakdown / non-finite value";
        case MPG_ERR_RANGE: return "value outside the storage precision's range";
        default: return "unknown mpgmres status";
    }
}

const char* mpg_ctx_last_error(mpg_ctx_t ctx) {
    return ctx ? ctx->last_error.c_str() : "null context";
}

int mpg_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int mpg_ctx_create(int device, mpg_ctx_t* out) {
    if (!out) return MPG_ERR_ARG;
    *out = nullptr;
    mpg_ctx* ctx = new (std::nothrow) mpg_ctx();
    if (!ctx) return MPG_ERR_ALLOC;
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) {
        ctx->red_ws_elems = mpg::kWsElems;
        e = hipMalloc(&ctx->red_ws, ctx->red_ws_elems * sizeof(double));
    }
    // coherent (fine-grained): the host polls words that kernels store while
    // they run (mpg::host_poll); the default kind if that is refused
    if (e == hipSuccess && hipHostMalloc(&ctx->host_ws, mpg::kHostWsBytes + 64, hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        ctx->host_ws = nullptr;
        e = hipHostMalloc(&ctx->host_ws, mpg::kHostWsBytes + 64, hipHostMallocDefault);
    }
    if (e == hipSuccess) std::memset(ctx->host_ws, 0, mpg::kHostWsBytes + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->ticket, 256);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->ticket, 0, 256, ctx->stream);
    if (e == hipSuccess && hipHostGetDevicePointer(&ctx->host_ws_dev, ctx->host_ws, 0) != hipSuccess) {
        ctx->host_ws_dev = nullptr;  // no device mapping: reductions copy their result out instead
        (void)hipGetLastError();
    }
    if (e != hipSuccess) {
        if (ctx->ticket) (void)hipFree(ctx->ticket);
        if (ctx->host_ws) (void)hipHostFree(ctx->host_ws);
        if (ctx->red_ws) (void)hipFree(ctx->red_ws);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return MPG_ERR_HIP;
    }
    *out = ctx;
    return MPG_OK;
}

int mpg_ctx_destroy(mpg_ctx_t ctx) {
    if (!ctx) return MPG_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->red_ws) (void)hipFree(ctx->red_ws);
    if (ctx->host_ws) (void)hipHostFree(ctx->host_ws);
    if (ctx->ticket) (void)hipFree(ctx->ticket);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return MPG_OK;
}

int mpg_ctx_sync(mpg_ctx_t ctx) {
    if (!ctx) return MPG_ERR_ARG;
    MPG_HIP(ctx, mpg::spin_wait(ctx->stream));
    return MPG_OK;
}

void* mpg_ctx_stream(mpg_ctx_t ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int mpg_ctx_device(mpg_ctx_t ctx) { return ctx ? ctx->device : -1; }

int mpg_malloc(mpg_ctx_t ctx, size_t bytes, void** out_dev) {
    if (!ctx || !out_dev) return MPG_ERR_ARG;
    *out_dev = nullptr;
    if (bytes == 0) return MPG_OK;
    // Round up to 256 B so vectorised kernels may touch whole 16-B granules.
    size_t padded = (bytes + 255) & ~size_t(255);
    hipError_t e = hipMalloc(out_dev, padded);
    if (e != hipSuccess) {
        mpg::set_hip_error(ctx, e, "hipMalloc");
        return MPG_ERR_ALLOC;
    }
    MPG_HIP(ctx, hipMemsetAsync(*out_dev, 0, padded, ctx->stream));
    return MPG_OK;
}

int mpg_free(mpg_ctx_t ctx, void* ptr_dev) {
    if (!ptr_dev) return MPG_OK;
    if (ctx) MPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    MPG_HIP(ctx, hipFree(ptr_dev));
    return MPG_OK;
}

int mpg_memset(mpg_ctx_t ctx, void* ptr_dev, int value, size_t bytes) {
    if (!ctx) return MPG_ERR_ARG;
    if (bytes == 0) return MPG_OK;
    MPG_HIP(ctx, hipMemsetAsync(ptr_dev, value, bytes, ctx->stream));
    return MPG_OK;
}

int mpg_memcpy_h2d(mpg_ctx_t ctx, void* dst_dev, const void* src_host, size_t bytes) {
    if (!ctx) return MPG_ERR_ARG;
    if (bytes == 0) return MPG_OK;
    if (bytes <= mpg::kHostWsBytes && ctx->host_ws) {  // small writes: pinned staging + a polled wait
        std::memcpy(ctx->host_ws, src_host, bytes);
        MPG_HIP(ctx, hipMemcpyAsync(dst_dev, ctx->host_ws, bytes, hipMemcpyHostToDevice, ctx->stream));
        MPG_HIP(ctx, mpg::spin_wait(ctx->stream));
        return MPG_OK;
    }
    MPG_HIP(ctx, hipMemcpyAsync(dst_dev, src_host, bytes, hipMemcpyHostToDevice, ctx->stream));
    // The host buffer may be pageable and reused by the caller right away.
    MPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MPG_OK;
}

int mpg_memcpy_d2h(mpg_ctx_t ctx, void* dst_host, const void* src_dev, size_t bytes) {
    if (!ctx) return MPG_ERR_ARG;
    if (bytes == 0) return MPG_OK;
    if (bytes <= mpg::kHostWsBytes && ctx->host_ws) {  // small reads: pinned staging + a polled wait
        if (ctx->host_ws_dev && bytes % 4 == 0 && (uintptr_t)src_dev % 4 == 0 && d2h_kernel()) {
            const bool poll = mpg::host_poll_on();
            const unsigned seq = poll ? mpg::host_seq_next(ctx) : 0u;
            k_d2h_words<<<1, 256, 0, ctx->stream>>>(static_cast<const uint32_t*>(src_dev),
                                                   static_cast<uint32_t*>(ctx->host_ws_dev), (int)(bytes / 4),
                                                   poll ? mpg::host_flag_dev(ctx) : nullptr, seq);
            MPG_HIP(ctx, hipGetLastError());
            if (poll) {
                MPG_HIP(ctx, mpg::host_poll(ctx, seq));
                std::memcpy(dst_host, ctx->host_ws, bytes);
                return MPG_OK;
            }
        } else {
            MPG_HIP(ctx, hipMemcpyAsync(ctx->host_ws, src_dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
        }
        MPG_HIP(ctx, mpg::spin_wait(ctx->stream));
        std::memcpy(dst_host, ctx->host_ws, bytes);
        return MPG_OK;
    }
    MPG_HIP(ctx, hipMemcpyAsync(dst_host, src_dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    MPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MPG_OK;
}

struct mpg_graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

int mpg_ctx_record_begin(mpg_ctx_t ctx) {
    if (!ctx) return MPG_ERR_ARG;
    MPG_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    return MPG_OK;
}

int mpg_ctx_record_end(mpg_ctx_t ctx, mpg_graph_t* out) {
    if (!ctx || !out) return MPG_ERR_ARG;
    *out = nullptr;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    (void)hipGetLastError();  // a void recording leaves its error sticky
    if (e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        return mpg::set_hip_error(ctx, e != hipSuccess ? e : hipErrorStreamCaptureInvalidated, "hipStreamEndCapture");
    }
    mpg_graph* p = new (std::nothrow) mpg_graph();
    if (!p) {
        (void)hipGraphDestroy(g);
        return MPG_ERR_ALLOC;
    }
    p->graph = g;
    const hipError_t ei = hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
        (void)hipGraphDestroy(g);
        delete p;
        return mpg::set_hip_error(ctx, ei, "hipGraphInstantiate");
    }
    *out = p;
    return MPG_OK;
}

int mpg_ctx_recording(mpg_ctx_t ctx) {
    if (!ctx) return 0;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(ctx->stream, &st) != hipSuccess) return 0;
    return st == hipStreamCaptureStatusActive ? 1 : 0;
}

int mpg_graph_launch(mpg_ctx_t ctx, mpg_graph_t g) {
    if (!ctx || !g || !g->exec) return MPG_ERR_ARG;
    MPG_HIP(ctx, hipGraphLaunch(g->exec, ctx->stream));
    return MPG_OK;
}

int mpg_graph_destroy(mpg_graph_t g) {
    if (!g) return MPG_OK;
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
    return MPG_OK;
}

int mpg_memcpy_d2d(mpg_ctx_t ctx, void* dst_dev, const void* src_dev, size_t bytes) {
    if (!ctx) return MPG_ERR_ARG;
    if (bytes == 0) return MPG_OK;
    MPG_HIP(ctx, hipMemcpyAsync(dst_dev, src_dev, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return MPG_OK;
}

}  // extern "C"
