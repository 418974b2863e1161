// api.hip — handle lifetime, error reporting and scratch management of libpcgpu.so.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "handle.h"

int pcg_fail(pcg_handle *h, int code, const char *fmt, ...) {
    if (h) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return code;
}

bool pcg_ensure(pcg_handle *h, DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return true;
    if (b.p) {
        hipStreamSynchronize(h->stream);
        hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    const size_t want = bytes + bytes / 8;  // headroom for the next level / call
    ++h->alloc_events;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        b.p = nullptr;
        return false;
    }
    b.bytes = want;
    return true;
}

bool pcg_ensure_pinned(pcg_handle *h, PinBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return true;
    if (b.p) {
        hipStreamSynchronize(h->stream);
        hipHostFree(b.p);
        b.p = nullptr;
        b.dp = nullptr;
        b.bytes = 0;
    }
    ++h->alloc_events;
    if (hipHostMalloc(&b.p, bytes, hipHostMallocMapped) != hipSuccess) {   // device-readable (k_copy_i64)
        b.p = nullptr;
        return false;
    }
    if (hipHostGetDevicePointer(&b.dp, b.p, 0) != hipSuccess) {   // once per allocation, not per level
        hipHostFree(b.p);
        b.p = b.dp = nullptr;
        return false;
    }
    b.bytes = bytes;
    return true;
}

extern "C" int pcg_abi_info(int64_t *stats_bytes, int64_t *record_bytes, int32_t *version) {
    if (stats_bytes) *stats_bytes = (int64_t)sizeof(pcg_stats);
    if (record_bytes) *record_bytes = (int64_t)sizeof(pcg_record);
    if (version) *version = PCG_ABI_VERSION;
    return PCG_OK;
}

namespace {
struct TuneSpec {
    const char *env;
    int64_t dflt, lo, hi;
};
// the knobs of pcgpu.h (PCG_TUNE_*): environment name, built-in value, accepted range
const TuneSpec kTune[PCG_TUNE_COUNT] = {
    {"PCG_SMALL", 1, 0, 1},
    {"PCG_SMALL_QCAP", 1024, 1, 1024},
    {"PCG_LDS_DEEP", 20, 12, 20},
    {"PCG_LDS_SPILL_MIN", 10000000, 0, INT64_MAX},
    {"PCG_WAVE_LO", 0, 0, PCG_MAX_LEVEL_DEPTH + 1},
    {"PCG_SCREEN_MASK", -1, -1, 0x1c},
    {"PCG_NODE_BLOCKS", 0x10, 0, 0x1c},
    {"PCG_EXPORT_INLINE", 16384, 0, INT64_MAX},
    {"PCG_NB", 0, 0, 1 << 24},
    {"PCG_NBW", 512, 1, 1 << 24},
    {"PCG_HOST_TRACE", 0, 0, 1},
    {"PCG_K1_I8", 1, 0, 1},
    {"PCG_K1_CRT", 1, 0, 1},
    {"PCG_K1_CRT_MINN", 256, 1, 1 << 24},
    {"PCG_K1_CRT_BITS", 53, 32, 63},
    {"PCG_K1_CRT_KS", 0, 0, 16},
    {"PCG_K1_I8_KS", 0, 0, 256},
    {"PCG_K1_SUPER_ORDER", 1, 0, 1},
    {"PCG_L1Z", 1, 0, 1},
};
}  // namespace

// read once, at pcg_create. A value pcg_set_tuning would refuse (not a whole base-0 integer, or
// outside the knob's range) keeps the built-in default and is reported on stderr, so a typo in an
// A/B knob never silently changes a plan or a launch shape
void pcg_tuning_defaults(int64_t *tune) {
    for (int k = 0; k < PCG_TUNE_COUNT; ++k) {
        int64_t v = kTune[k].dflt;
        if (const char *e = getenv(kTune[k].env)) {
            char *end = nullptr;
            errno = 0;
            const long long p = strtoll(e, &end, 0);
            if (end == e || *end != '\0' || errno == ERANGE || p < kTune[k].lo || p > kTune[k].hi)
                fprintf(stderr, "pcgpu: ignoring %s=%s (not an integer in [%lld, %lld]); using %lld\n", kTune[k].env, e,
                        (long long)kTune[k].lo, (long long)kTune[k].hi, (long long)kTune[k].dflt);
            else
                v = p;
        }
        tune[k] = v;
    }
}

extern "C" int pcg_set_tuning(pcg_handle *h, int key, int64_t value) {
    if (!h || key < 0 || key >= PCG_TUNE_COUNT || value < kTune[key].lo || value > kTune[key].hi)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_tuning: key %d value %lld", key, (long long)value);
    h->tune[key] = value;
    return PCG_OK;
}

extern "C" int pcg_get_tuning(pcg_handle *h, int key, int64_t *value) {
    if (!h || !value || key < 0 || key >= PCG_TUNE_COUNT)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_get_tuning: key %d", key);
    *value = h->tune[key];
    return PCG_OK;
}

extern "C" int pcg_create(int device, pcg_handle **out) {
    if (!out) return PCG_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PCG_ERR_HIP;
    if (device < 0 || device >= ndev) return PCG_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return PCG_ERR_HIP;
    pcg_handle *h = new pcg_handle();
    h->device = device;
    pcg_tuning_defaults(h->tune);
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return PCG_ERR_HIP;
    }
    h->own_stream = true;
    for (auto &e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) {
            delete h;
            return PCG_ERR_HIP;
        }
    *out = h;
    return PCG_OK;
}

extern "C" int pcg_destroy(pcg_handle *h) {
    if (!h) return PCG_OK;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    pcg_comm_release(h);
    if (h->xs) hipStreamSynchronize(h->xs);
    DevBuf *bufs[] = {&h->adj, &h->deg, &h->off2[0], &h->off2[1], &h->nbr2[0], &h->nbr2[1], &h->rm, &h->ug2[0],
                      &h->ug2[1], &h->exp_ctr, &h->cpre, &h->binom, &h->ctr,
                      &h->deferred, &h->screenq, &h->records, &h->nearbuf, &h->exportbuf, &h->export_xy, &h->diag,
                      &h->colmean, &h->pr_scratch, &h->batch_scratch, &h->chisq_scratch, &h->cblk, &h->lmk,
                      &h->k1_digits, &h->small_sum};
    for (DevBuf *b : bufs)
        if (b->p) hipFree(b->p);
    PinBuf *pins[] = {&h->ctr_pin, &h->deg_pin, &h->off_pin, &h->cpre_pin, &h->status_pin, &h->small_pin, &h->near_pin};
    for (PinBuf *b : pins)
        if (b->p) hipHostFree(b->p);
    if (h->summary) hipHostFree(h->summary);
    for (auto &e : h->ev)
        if (e) hipEventDestroy(e);
    for (auto &e : h->lev)
        if (e) hipEventDestroy(e);
    for (auto &pr : h->rev)
        for (auto &e : pr)
            if (e) hipEventDestroy(e);
    if (h->ev_join) hipEventDestroy(h->ev_join);
    if (h->ev_fork) hipEventDestroy(h->ev_fork);
    if (h->tail) hipHostFree(h->tail);
    if (h->aux) hipStreamDestroy(h->aux);
    if (h->xs) hipStreamDestroy(h->xs);
    if (h->ev_xready) hipEventDestroy(h->ev_xready);
    for (auto &e : h->ev_xdone)
        if (e) hipEventDestroy(e);
    if (h->own_stream && h->stream) hipStreamDestroy(h->stream);
    delete h;
    return PCG_OK;
}

extern "C" const char *pcg_last_error(pcg_handle *h) { return h ? h->err.c_str() : "null handle"; }

extern "C" int pcg_set_stream(pcg_handle *h, void *hip_stream) {
    if (!h) return PCG_ERR_INVALID;
    hipStreamSynchronize(h->stream);
    if (h->own_stream && h->stream) hipStreamDestroy(h->stream);
    // NULL is the default stream itself (not "make one"): torch's default current stream
    // reports handle 0, and a private non-blocking stream would not be ordered after torch's
    // writes to the buffers handed over
    h->stream = (hipStream_t)hip_stream;
    h->own_stream = false;
    return PCG_OK;
}

extern "C" int pcg_set_capacity(pcg_handle *h, int64_t record_capacity, int64_t deferred_capacity) {
    if (!h) return PCG_ERR_INVALID;
    if (record_capacity > 0) h->rec_cap = record_capacity;
    if (deferred_capacity > 0) h->def_cap = deferred_capacity;
    return PCG_OK;
}

extern "C" int pcg_set_screen_capacity(pcg_handle *h, int64_t entries) {
    if (!h || entries < 1) return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_screen_capacity: %lld", (long long)entries);
    h->scr_cap = entries;
    return PCG_OK;
}

extern "C" int pcg_set_record_sample(pcg_handle *h, int64_t modulus, int64_t residue) {
    if (!h || modulus < 0 || (modulus > 1 && (residue < 0 || residue >= modulus)))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_record_sample: modulus %lld residue %lld", (long long)modulus,
                        (long long)residue);
    h->rec_mod = modulus;
    h->rec_res = residue;
    return PCG_OK;
}
