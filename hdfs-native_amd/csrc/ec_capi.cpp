// ec_capi.cpp -- implementation of the C ABI in include/hdfs_ec_amd.h.
//
// Host-side logic of hdfs-native's Coder (rust/src/ec/gf256.rs:25-138) on top
// of the HIP kernels in ec_kernels.hip:
//   * coding matrix (gen_rs_matrix, gf256.rs:40-57) built once per coder;
//   * decode plans (first-k-present survivors, inverse, missing-data rows;
//     gf256.rs:84-126) computed once per erasure mask and cached -- the
//     reference rebuilds Coder and re-inverts per decoded row (ec/mod.rs:71);
//   * host-buffer calls stage through coder-owned device buffers;
//   * device calls only enqueue kernels on the caller's stream.
// Nothing here throws or aborts across the ABI: every entry point catches.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <fstream>
#include <map>
#include <tuple>
#include <memory>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <new>
#include <unordered_map>
#include <vector>

#include "../../include/hdfs_ec_amd.h"
#include "../../include/hdfs_ec_amd_exp.h"
#include "checksum.hpp"
#include "checksum_tables.hpp"
#include "ec_kernels.hpp"
#include "gf256.hpp"
#include "host_gf.hpp"
#include "jit.hpp"

namespace {

thread_local char g_last_error[256] = "";

// Records the failing HIP call for hec_last_error() and returns `status`.
int fail(int status, const char* what, hipError_t err) {
    std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s (%d)", what, hipGetErrorString(err), int(err));
    return status;
}

#define HEC_HIP(call, status)                                  \
    do {                                                       \
        hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) {                                \
            (void)hipGetLastError();                           \
            return fail((status), #call, e_);                  \
        }                                                      \
    } while (0)

struct DecodePlan {
    int status = HEC_OK;
    std::vector<size_t> survivors;  // k
    std::vector<size_t> missing;    // e
    std::vector<uint8_t> matrix;    // e x k
    std::vector<uint32_t> perm;     // e x k x 8: the matrix's v_perm product tables (mixed-decode plan blobs)
    std::vector<uint64_t> aff;      // e x k: the matrix's host affine qwords (small-row host path)
};

// Restores the caller's current HIP device on scope exit.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (dev < 0) return;  // a host-only coder (HEC_DEVICE_HOST): no device, no HIP call
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct hec_coder {
    size_t k = 0, m = 0;
    int device = 0;
    bool xor_codec = false;
    std::string codec;         // "rs", "xor" or "rs-legacy"
    bool pooled = false;       // handed out by hec_coder_acquire (returned by hec_coder_release)
    bool idle = false;         // pooled and sitting in the pool (guarded by the pool mutex)
    std::vector<uint8_t> enc;  // (k+m) x k
    std::vector<uint64_t> enc_aff;  // m x k: host affine qwords of the parity rows
    // hec_encode / hec_decode rows of at most this many bytes per shard are
    // coded on the host (hec::host), larger ones go through the device
    std::atomic<size_t> host_limit{kDefaultHostLimit};
    // Every row on pageable buffers: the host routine beat the device route at
    // every size measured, cold (rows from a 1 GiB pool) and hot, 4 KiB to
    // 4 MiB per shard (profiles/r04d/); set a limit to route
    // longer rows through the device.
    static constexpr size_t kDefaultHostLimit = SIZE_MAX;

    // Decode plans keyed by presence bitmask (k+m <= 48), bounded: at most
    // kPlanCacheMax entries; past that the least recently used eighth is
    // dropped (mixed and verified reads can feed it any mask).  Entries are
    // shared_ptrs, so a plan a caller still holds outlives its eviction.
    static constexpr size_t kPlanCacheMax = 4096;
    struct PlanSlot {
        std::shared_ptr<const DecodePlan> plan;
        uint64_t last_use;
    };
    std::mutex plan_mu;
    std::unordered_map<uint64_t, PlanSlot> plans;
    uint64_t plan_clock = 0;

    std::mutex host_mu;  // serialises the host-buffer API (staging buffers)
    static constexpr int kSlots = 3;
    hipStream_t stream = nullptr;                       // compute
    hipStream_t copy_stream[2] = {nullptr, nullptr};    // [0] H2D, [1] D2H
    hipEvent_t ev_in[kSlots] = {}, ev_k[kSlots] = {}, ev_out[kSlots] = {};
    uint8_t* dbuf = nullptr;
    size_t dbuf_bytes = 0;
    // hec_encode / hec_decode (one row per call, pageable caller buffers):
    // a persistent pinned bounce buffer and device slots of their own, grown
    // geometrically and released only by hec_coder_destroy
    static constexpr int kCallPieces = 16;  // column pieces of one per-call row (pipeline stages)
    static constexpr int kCallEvents = 3 * kCallPieces;
    uint8_t* call_host = nullptr;  // hipHostMalloc'd
    uint8_t* call_dev = nullptr;
    size_t call_bytes = 0;
    hipEvent_t ev_call[kCallEvents] = {};
    // verified read, phase 2: stripe lists + mixed-decode workspace (device),
    // grown geometrically, released by hec_coder_destroy.  verify_mu is held
    // from the first list upload until the holder's stream has drained, so two
    // threads verifying on one coder never share (or free) it under each
    // other's queued work.
    std::mutex verify_mu;
    uint8_t* verify_ws = nullptr;
    size_t verify_ws_bytes = 0;
    // mixed decode: two pinned staging images for the workspace upload (so
    // the H2D is a real async DMA), each reused once its copy has run
    std::mutex mixed_mu;
    uint8_t* mixed_host[2] = {nullptr, nullptr};
    size_t mixed_host_bytes[2] = {0, 0};
    hipEvent_t ev_mixed[2] = {nullptr, nullptr};
    int mixed_next = 0;
};

namespace {

// launch_gf_matmul: 0 ok, -1 invalid sizes, >0 the hipError_t of the launch.
int to_status(int kernel_rc) {
    if (kernel_rc == 0) return HEC_OK;
    if (kernel_rc == -1) return HEC_ERR_INVALID_ARG;
    return fail(HEC_ERR_DEVICE, "kernel launch", hipError_t(kernel_rc));
}

DecodePlan compute_plan(size_t k, size_t m, const uint8_t* present, const std::vector<uint8_t>& enc) {
    DecodePlan p;
    std::vector<size_t> valid;
    for (size_t i = 0; i < k + m; i++) {
        if (present[i])
            valid.push_back(i);
        else if (i < k)
            p.missing.push_back(i);  // gf256.rs:96-97: only data indices
    }
    if (p.missing.empty()) return p;  // gf256.rs:102-105
    if (valid.size() < k) {           // gf256.rs:107-111
        p.status = HEC_ERR_NOT_ENOUGH_SHARDS;
        return p;
    }
    p.survivors.assign(valid.begin(), valid.begin() + k);  // first k present, ascending
    std::vector<uint8_t> sub(k * k);
    for (size_t r = 0; r < k; r++) std::memcpy(&sub[r * k], &enc[p.survivors[r] * k], k);  // select_rows
    if (!hec::invert(sub.data(), k)) {
        p.status = HEC_ERR_SINGULAR;
        return p;
    }
    p.matrix.resize(p.missing.size() * k);
    for (size_t r = 0; r < p.missing.size(); r++)  // select_rows(invalid), ascending
        std::memcpy(&p.matrix[r * k], &sub[p.missing[r] * k], k);
    p.perm.resize(p.matrix.size() * 8);
    for (size_t x = 0; x < p.matrix.size(); x++) {
        const auto w = hec::perm_table_words(p.matrix[x]);
        std::memcpy(&p.perm[x * 8], w.data(), sizeof(uint32_t) * 8);
    }
    p.aff = hec::host::affine_matrices(p.matrix.data(), p.matrix.size());
    return p;
}

using PlanRef = std::shared_ptr<const DecodePlan>;

PlanRef cached_plan(hec_coder* c, const uint8_t* present) {
    uint64_t key = 0;
    for (size_t i = 0; i < c->k + c->m; i++)
        if (present[i]) key |= uint64_t(1) << i;
    std::lock_guard<std::mutex> lk(c->plan_mu);
    const uint64_t now = ++c->plan_clock;
    auto it = c->plans.find(key);
    if (it != c->plans.end()) {
        it->second.last_use = now;
        return it->second.plan;
    }
    if (c->plans.size() >= hec_coder::kPlanCacheMax) {
        // evict the least recently used eighth (one pass to find the cut)
        std::vector<uint64_t> uses;
        uses.reserve(c->plans.size());
        for (const auto& kv : c->plans) uses.push_back(kv.second.last_use);
        const size_t n_evict = c->plans.size() / 8;
        std::nth_element(uses.begin(), uses.begin() + n_evict, uses.end());
        const uint64_t cut = uses[n_evict];
        for (auto e = c->plans.begin(); e != c->plans.end();)
            e = e->second.last_use < cut ? c->plans.erase(e) : std::next(e);
    }
    PlanRef p = std::make_shared<const DecodePlan>(compute_plan(c->k, c->m, present, c->enc));
    c->plans.emplace(key, hec_coder::PlanSlot{p, now});
    return p;
}

// Runs out[j] = sum_i mat[j*cols+i] * in[i] over a batch, <= 4 rows per launch.
int matmul_batch(int device, const uint8_t* mat, size_t rows, size_t cols, const uint8_t* const* in,
                 const size_t* in_strides, uint8_t* const* out, const size_t* out_strides, size_t cell_len,
                 size_t stripes, hipStream_t stream) {
    if (rows == 0 || cols == 0 || cols > size_t(hec::kMaxK) || cell_len == 0 || !mat || !in || !out ||
        !in_strides || !out_strides)
        return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    for (size_t i = 0; i < cols; i++)
        if (!in[i]) return HEC_ERR_INVALID_ARG;
    for (size_t j = 0; j < rows; j++)
        if (!out[j]) return HEC_ERR_INVALID_ARG;
    for (size_t r0 = 0; r0 < rows; r0 += hec::kMaxR) {
        hec::MatmulArgs a;
        std::memset(&a, 0, sizeof(a));
        const size_t nr = std::min(rows - r0, size_t(hec::kMaxR));
        for (size_t i = 0; i < cols; i++) {
            a.in[i] = in[i];
            a.in_stride[i] = in_strides[i];
        }
        for (size_t j = 0; j < nr; j++) {
            a.out[j] = out[r0 + j];
            a.out_stride[j] = out_strides[r0 + j];
            for (size_t i = 0; i < cols; i++) a.coef[j * hec::kMaxK + i] = mat[(r0 + j) * cols + i];
        }
        a.k = int32_t(cols);
        a.r = int32_t(nr);
        a.cell_len = cell_len;
        a.stripes = stripes;
        const int rc = hec::launch_gf_matmul(a, device, stream);
        if (rc != 0) return to_status(rc);
    }
    return HEC_OK;
}

// Drains the coder's three streams on scope exit, errors ignored: a pipeline
// that fails half-way never returns while its DMA still reads or writes the
// caller's host buffers (or the slot buffers the next call may reallocate).
struct StreamDrain {
    hec_coder* c;
    ~StreamDrain() {
        (void)hipStreamSynchronize(c->copy_stream[0]);
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->copy_stream[1]);
        (void)hipGetLastError();
    }
};

// Grows the per-call staging (pinned host + device) to `bytes`, doubling so
// that a stream of growing rows reallocates O(log) times; never shrinks.
int ensure_call_staging(hec_coder* c, size_t bytes) {
    if (c->call_bytes >= bytes) return HEC_OK;
    const size_t want = std::max(bytes, c->call_bytes * 2);
    if (c->call_host) (void)hipHostFree(c->call_host);
    if (c->call_dev) (void)hipFree(c->call_dev);
    c->call_host = c->call_dev = nullptr;
    c->call_bytes = 0;
    HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->call_host), want, hipHostMallocDefault), HEC_ERR_NO_MEMORY);
    HEC_HIP(hipMalloc(&c->call_dev, want), HEC_ERR_NO_MEMORY);
    c->call_bytes = want;
    return HEC_OK;
}

// One row through the device, pageable caller buffers in and out:
//   out[j] = sum_i mat[j*nin + i] * in[i], n bytes each.
// Rows of >= 512 KiB are cut into column pieces (>= 256 KiB of every shard,
// at most kCallPieces) that flow through a three-stage pipeline: the
// caller's thread copies piece p of every input into the pinned bounce
// buffer and queues its H2D (one 2D copy on copy_stream[0]); the compute
// stream runs the kernel on piece p once it has landed; copy_stream[1]
// brings piece p of the outputs back (one 2D copy) and the caller copies it
// out.  Host copies, both PCIe directions and the kernel then overlap within
// one call.  Smaller rows go through in one piece, one DMA each way.
// No allocation on the hot path.
int call_through_device(hec_coder* c, const uint8_t* const* in, size_t nin, uint8_t* const* out, size_t nout,
                        const uint8_t* mat, size_t n) {
    const size_t pitch = (n + 255) & ~size_t(255);
    int rc = ensure_call_staging(c, pitch * (nin + nout));
    if (rc != HEC_OK) return rc;
    StreamDrain drain{c};  // never return with a DMA still touching the bounce buffer
    const uint8_t* din[HEC_MAX_DATA_UNITS];
    uint8_t* dout[HEC_MAX_DATA_UNITS];
    size_t strides[HEC_MAX_DATA_UNITS];
    for (size_t i = 0; i < std::max(nin, nout); i++) strides[i] = pitch;
    uint8_t* hin = c->call_host;
    uint8_t* hout = c->call_host + nin * pitch;
    uint8_t* dinb = c->call_dev;
    uint8_t* doutb = c->call_dev + nin * pitch;

    const int piece_kib = hec::tune_snapshot().call_piece_kib;  // tune key 17 (0 = 256 KiB)
    const size_t kMinPiece = size_t(piece_kib > 0 ? piece_kib : 256) << 10;
    if (n >= 2 * kMinPiece) {
        size_t piece = (n + hec_coder::kCallPieces - 1) / hec_coder::kCallPieces;
        piece = std::max(kMinPiece, (piece + 4095) & ~size_t(4095));
        const size_t pieces = (n + piece - 1) / piece;
        hipStream_t h2d = c->copy_stream[0], d2h = c->copy_stream[1];
        hipEvent_t* ev_in = c->ev_call;
        hipEvent_t* ev_k = c->ev_call + hec_coder::kCallPieces;
        hipEvent_t* ev_out = c->ev_call + 2 * hec_coder::kCallPieces;
        for (size_t q = 0; q < pieces; q++) {
            const size_t off = q * piece, len = std::min(piece, n - off);
            for (size_t i = 0; i < nin; i++) std::memcpy(hin + i * pitch + off, in[i] + off, len);
            HEC_HIP(hipMemcpy2DAsync(dinb + off, pitch, hin + off, pitch, len, nin, hipMemcpyHostToDevice, h2d),
                    HEC_ERR_DEVICE);
            HEC_HIP(hipEventRecord(ev_in[q], h2d), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamWaitEvent(c->stream, ev_in[q], 0), HEC_ERR_DEVICE);
            for (size_t i = 0; i < nin; i++) din[i] = dinb + i * pitch + off;
            for (size_t j = 0; j < nout; j++) dout[j] = doutb + j * pitch + off;
            rc = matmul_batch(c->device, mat, nout, nin, din, strides, dout, strides, len, 1, c->stream);
            if (rc != HEC_OK) return rc;
            HEC_HIP(hipEventRecord(ev_k[q], c->stream), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamWaitEvent(d2h, ev_k[q], 0), HEC_ERR_DEVICE);
            HEC_HIP(hipMemcpy2DAsync(hout + off, pitch, doutb + off, pitch, len, nout, hipMemcpyDeviceToHost, d2h),
                    HEC_ERR_DEVICE);
            HEC_HIP(hipEventRecord(ev_out[q], d2h), HEC_ERR_DEVICE);
        }
        for (size_t q = 0; q < pieces; q++) {
            const size_t off = q * piece, len = std::min(piece, n - off);
            HEC_HIP(hipEventSynchronize(ev_out[q]), HEC_ERR_DEVICE);
            for (size_t j = 0; j < nout; j++) std::memcpy(out[j] + off, hout + j * pitch + off, len);
        }
        return HEC_OK;
    }

    // one piece: one DMA each way on the compute stream (fewer, larger copies
    // beat per-shard ones below 512 KiB: profiles/r02_probe_percall*.log)
    for (size_t i = 0; i < nin; i++) {
        std::memcpy(hin + i * pitch, in[i], n);
        din[i] = dinb + i * pitch;
    }
    HEC_HIP(hipMemcpyAsync(dinb, hin, pitch * (nin - 1) + n, hipMemcpyHostToDevice, c->stream), HEC_ERR_DEVICE);
    for (size_t j = 0; j < nout; j++) dout[j] = doutb + j * pitch;
    rc = matmul_batch(c->device, mat, nout, nin, din, strides, dout, strides, n, 1, c->stream);
    if (rc != HEC_OK) return rc;
    HEC_HIP(hipMemcpyAsync(hout, doutb, pitch * (nout - 1) + n, hipMemcpyDeviceToHost, c->stream), HEC_ERR_DEVICE);
    HEC_HIP(hipStreamSynchronize(c->stream), HEC_ERR_DEVICE);
    for (size_t j = 0; j < nout; j++) std::memcpy(out[j], hout + j * pitch, n);
    return HEC_OK;
}

// One row of pageable host buffers, routed by size: rows of at most the
// coder's host limit are coded on this thread (hec::host, no lock), larger
// ones through the device under the coder's host lock.
int code_row(hec_coder* c, const uint8_t* mat, const uint64_t* aff, const uint8_t* const* in, size_t nin,
             uint8_t* const* out, size_t nout, size_t n) {
    if (c->device == HEC_DEVICE_HOST || n <= c->host_limit.load(std::memory_order_relaxed)) {
        hec::host::gf_matmul_split(mat, aff, nout, nin, in, out, n);
        return HEC_OK;
    }
    std::lock_guard<std::mutex> lk(c->host_mu);
    DeviceGuard g(c->device);
    if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
    return call_through_device(c, in, nin, out, nout, mat, n);
}

int ensure_dbuf(hec_coder* c, size_t bytes) {
    if (c->dbuf_bytes >= bytes) return HEC_OK;
    if (c->dbuf) (void)hipFree(c->dbuf);
    c->dbuf = nullptr;
    c->dbuf_bytes = 0;
    HEC_HIP(hipMalloc(&c->dbuf, bytes), HEC_ERR_NO_MEMORY);
    c->dbuf_bytes = bytes;
    return HEC_OK;
}

// Device-resident calls on a host-only coder (HEC_DEVICE_HOST): an error, never
// a HIP call.
int host_only(const char* what) { return fail(HEC_ERR_DEVICE, what, hipErrorNoDevice); }

template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return HEC_ERR_NO_MEMORY;
    } catch (...) {
        return fail(HEC_ERR_DEVICE, "unexpected C++ exception", hipErrorUnknown);
    }
}

}  // namespace

extern "C" {

const char* hec_strerror(int status) {
    switch (status) {
        case HEC_OK: return "ok";
        case HEC_ERR_INVALID_ARG: return "invalid argument";
        case HEC_ERR_NOT_ENOUGH_SHARDS: return "erasure coding error: Not enough valid shards";
        case HEC_ERR_UNSUPPORTED_CODEC: return "unsupported erasure coding policy";
        case HEC_ERR_DEVICE: return "HIP device error";
        case HEC_ERR_NO_MEMORY: return "out of memory";
        case HEC_ERR_SINGULAR: return "Matrix is singular";
        case HEC_ERR_CHECKSUM: return "checksum error";
        default: return "unknown status";
    }
}

int hec_abi_version(void) { return HEC_ABI_VERSION; }

const char* hec_last_error(void) { return g_last_error; }

int hec_gen_rs_matrix(size_t data_units, size_t parity_units, uint8_t* out) {
    if (!out || data_units == 0 || data_units + parity_units > 256) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        const std::vector<uint8_t> m = hec::gen_rs_matrix(data_units, parity_units);
        std::memcpy(out, m.data(), m.size());
        return HEC_OK;
    });
}

int hec_gen_codec_matrix(const char* codec, size_t data_units, size_t parity_units, uint8_t* out) {
    if (!out || data_units == 0 || parity_units == 0 || data_units + parity_units > 255) return HEC_ERR_INVALID_ARG;
    const std::string name = codec ? codec : "rs";
    if (name != "rs" && name != "xor" && name != "rs-legacy") return HEC_ERR_UNSUPPORTED_CODEC;
    if (name == "xor" && parity_units != 1) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        const std::vector<uint8_t> m = name == "xor"         ? hec::gen_xor_matrix(data_units)
                                       : name == "rs-legacy" ? hec::gen_rs_legacy_matrix(data_units, parity_units)
                                                             : hec::gen_rs_matrix(data_units, parity_units);
        std::memcpy(out, m.data(), m.size());
        return HEC_OK;
    });
}

int hec_matrix_invert(uint8_t* mat, size_t n) {
    if (!mat || n == 0) return HEC_ERR_INVALID_ARG;
    return guarded([&] { return hec::invert(mat, n) ? HEC_OK : HEC_ERR_SINGULAR; });
}

int hec_decode_plan(size_t data_units, size_t parity_units, const uint8_t* present, size_t* n_missing,
                    size_t* survivors, size_t* missing, uint8_t* matrix) {
    if (!present || !n_missing || data_units == 0 || parity_units == 0 || data_units + parity_units > 256)
        return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        DecodePlan p = compute_plan(data_units, parity_units, present, hec::gen_rs_matrix(data_units, parity_units));
        *n_missing = p.missing.size();
        if (p.status != HEC_OK) return p.status;
        if (survivors) std::copy(p.survivors.begin(), p.survivors.end(), survivors);
        if (missing) std::copy(p.missing.begin(), p.missing.end(), missing);
        if (matrix) std::copy(p.matrix.begin(), p.matrix.end(), matrix);
        return HEC_OK;
    });
}

int hec_coder_create_codec(const char* codec, size_t data_units, size_t parity_units, int device,
                           hec_coder_t** out) {
    if (!out) return HEC_ERR_INVALID_ARG;
    *out = nullptr;
    if (data_units == 0 || data_units > HEC_MAX_DATA_UNITS || parity_units == 0 ||
        parity_units > HEC_MAX_PARITY_UNITS)
        return HEC_ERR_INVALID_ARG;
    const std::string name = codec ? codec : "rs";
    if (name != "rs" && name != "xor" && name != "rs-legacy") return HEC_ERR_UNSUPPORTED_CODEC;
    if (name == "xor" && parity_units != 1) return HEC_ERR_INVALID_ARG;  // XOR-k-1 only
    return guarded([&] {
        if (device != HEC_DEVICE_HOST) {
            int ndev = 0;
            HEC_HIP(hipGetDeviceCount(&ndev), HEC_ERR_DEVICE);
            if (device < 0 || device >= ndev) return fail(HEC_ERR_DEVICE, "device ordinal", hipErrorInvalidDevice);
        }
        auto* c = new hec_coder();
        c->k = data_units;
        c->m = parity_units;
        c->device = device;
        c->xor_codec = name == "xor";
        c->codec = name;
        c->enc = c->xor_codec            ? hec::gen_xor_matrix(data_units)
                 : name == "rs-legacy" ? hec::gen_rs_legacy_matrix(data_units, parity_units)
                                       : hec::gen_rs_matrix(data_units, parity_units);
        c->enc_aff = hec::host::affine_matrices(c->enc.data() + data_units * data_units, parity_units * data_units);
        if (device == HEC_DEVICE_HOST) {  // host routine only: no stream, event or buffer
            c->host_limit.store(SIZE_MAX, std::memory_order_relaxed);
            *out = c;
            return int(HEC_OK);
        }
        int rc = [&] {
            DeviceGuard g(device);
            if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
            HEC_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), HEC_ERR_DEVICE);
            for (int i = 0; i < 2; i++)
                HEC_HIP(hipStreamCreateWithFlags(&c->copy_stream[i], hipStreamNonBlocking), HEC_ERR_DEVICE);
            for (int i = 0; i < hec_coder::kCallEvents; i++)
                HEC_HIP(hipEventCreateWithFlags(&c->ev_call[i], hipEventDisableTiming), HEC_ERR_DEVICE);
            for (int i = 0; i < hec_coder::kSlots; i++) {
                HEC_HIP(hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming), HEC_ERR_DEVICE);
                HEC_HIP(hipEventCreateWithFlags(&c->ev_k[i], hipEventDisableTiming), HEC_ERR_DEVICE);
                HEC_HIP(hipEventCreateWithFlags(&c->ev_out[i], hipEventDisableTiming), HEC_ERR_DEVICE);
            }
            hec::queue_reserve(device);  // graph-capture counter sets, outside any capture
            return HEC_OK;
        }();
        if (rc != HEC_OK) {
            hec_coder_destroy(c);
            return rc;
        }
        *out = c;
        return HEC_OK;
    });
}

int hec_coder_create(size_t data_units, size_t parity_units, int device, hec_coder_t** out) {
    return hec_coder_create_codec("rs", data_units, parity_units, device, out);
}

void hec_coder_destroy(hec_coder_t* c) {
    if (!c) return;
    try {
        DeviceGuard g(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        for (auto s : c->copy_stream)
            if (s) (void)hipStreamSynchronize(s);
        if (c->dbuf) (void)hipFree(c->dbuf);
        if (c->call_dev) (void)hipFree(c->call_dev);
        if (c->call_host) (void)hipHostFree(c->call_host);
        if (c->verify_ws) {  // stream-ordered allocation (verified read phase 2)
            (void)hipFreeAsync(c->verify_ws, nullptr);
            (void)hipStreamSynchronize(nullptr);
        }
        for (int i = 0; i < 2; i++) {
            if (c->ev_mixed[i]) (void)hipEventSynchronize(c->ev_mixed[i]);
            if (c->mixed_host[i]) (void)hipHostFree(c->mixed_host[i]);
            if (c->ev_mixed[i]) (void)hipEventDestroy(c->ev_mixed[i]);
        }
        for (hipEvent_t e : c->ev_call)
            if (e) (void)hipEventDestroy(e);
        for (int i = 0; i < hec_coder::kSlots; i++)
            for (hipEvent_t e : {c->ev_in[i], c->ev_k[i], c->ev_out[i]})
                if (e) (void)hipEventDestroy(e);
        for (auto s : c->copy_stream)
            if (s) (void)hipStreamDestroy(s);
        if (c->stream) (void)hipStreamDestroy(c->stream);
    } catch (...) {
    }
    delete c;
}

}  // extern "C"

// ---- coder pool: Coder::new per row (gf256.rs:32-38, ec/mod.rs:71) ----------

namespace {

// Idle coders by (codec, k, m, device).  hec_coder_acquire pops one (or
// creates one); hec_coder_release pushes it back, so a caller that builds a
// Coder per decoded row pays a mutex and a vector pop, not 3 streams, 60
// events and the staging buffers.  A coder is exclusively the acquirer's
// until it is released.  The pool is never destroyed (coders are not freed
// from a static destructor, after the HIP runtime may be gone).
struct CoderPool {
    std::mutex mu;
    std::map<std::tuple<std::string, size_t, size_t, int>, std::vector<hec_coder*>> idle;
    std::atomic<unsigned> next_device{0};
};
constexpr size_t kPoolIdlePerKey = 64;  // idle coders kept per key; more are destroyed on release

CoderPool& coder_pool() {
    static CoderPool* p = new CoderPool;
    return *p;
}

}  // namespace

extern "C" {

int hec_coder_acquire(const char* codec, size_t data_units, size_t parity_units, int device, hec_coder_t** out) {
    if (!out) return HEC_ERR_INVALID_ARG;
    *out = nullptr;
    if (device < HEC_DEVICE_HOST) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        const std::string name = codec ? codec : "rs";
        if (device == -1) {  // any device: round-robin over the visible ones; none -> host-only
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
                device = HEC_DEVICE_HOST;
            else
                device = int(coder_pool().next_device.fetch_add(1, std::memory_order_relaxed) % unsigned(ndev));
        }
        CoderPool& pool = coder_pool();
        {
            std::lock_guard<std::mutex> lk(pool.mu);
            auto it = pool.idle.find(std::make_tuple(name, data_units, parity_units, device));
            if (it != pool.idle.end() && !it->second.empty()) {
                *out = it->second.back();
                it->second.pop_back();
                (*out)->idle = false;
                return int(HEC_OK);
            }
        }
        hec_coder_t* c = nullptr;
        const int rc = hec_coder_create_codec(name.c_str(), data_units, parity_units, device, &c);
        if (rc != HEC_OK) return rc;
        c->pooled = true;
        *out = c;
        return int(HEC_OK);
    });
}

void hec_coder_release(hec_coder_t* c) {
    if (!c) return;
    if (c->pooled) {
        try {
            CoderPool& pool = coder_pool();
            std::lock_guard<std::mutex> lk(pool.mu);
            // a second release of a coder already in the pool is ignored: pushing
            // it twice would hand one coder to two "exclusive" acquirers
            if (c->idle) return;
            // the next acquirer gets a coder with default behaviour: a host
            // limit set by this user (e.g. 0 to force the device) does not carry over
            c->host_limit.store(c->device == HEC_DEVICE_HOST ? SIZE_MAX : hec_coder::kDefaultHostLimit,
                                std::memory_order_relaxed);
            auto& v = pool.idle[std::make_tuple(c->codec, c->k, c->m, c->device)];
            if (v.size() < kPoolIdlePerKey) {
                c->idle = true;
                v.push_back(c);
                return;
            }
        } catch (...) {
        }
    }
    hec_coder_destroy(c);
}

size_t hec_coder_pool_trim(void) {
    std::vector<hec_coder*> drop;
    try {
        CoderPool& pool = coder_pool();
        std::lock_guard<std::mutex> lk(pool.mu);
        for (auto& kv : pool.idle) drop.insert(drop.end(), kv.second.begin(), kv.second.end());
        pool.idle.clear();
    } catch (...) {
        return 0;
    }
    for (hec_coder* c : drop) hec_coder_destroy(c);
    return drop.size();
}

size_t hec_coder_data_units(const hec_coder_t* c) { return c ? c->k : 0; }
size_t hec_coder_parity_units(const hec_coder_t* c) { return c ? c->m : 0; }
int hec_coder_device(const hec_coder_t* c) { return c ? c->device : -1; }

int hec_coder_set_host_limit(hec_coder_t* c, size_t max_shard_len) {
    if (!c) return HEC_ERR_INVALID_ARG;
    c->host_limit.store(max_shard_len, std::memory_order_relaxed);
    return HEC_OK;
}

size_t hec_coder_host_limit(const hec_coder_t* c) { return c ? c->host_limit.load(std::memory_order_relaxed) : 0; }

const char* hec_host_isa(void) { return hec::host::isa_name(hec::host::best_isa()); }

int hec_gf_matmul_host(const uint8_t* matrix, size_t rows, size_t cols, const uint8_t* const* in, uint8_t* const* out,
                       size_t len) {
    if (!matrix || !in || !out || rows == 0 || cols == 0 || cols > HEC_MAX_DATA_UNITS || len == 0)
        return HEC_ERR_INVALID_ARG;
    for (size_t i = 0; i < cols; i++)
        if (!in[i]) return HEC_ERR_INVALID_ARG;
    for (size_t j = 0; j < rows; j++)
        if (!out[j]) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        hec::host::gf_matmul_split(matrix, nullptr, rows, cols, in, out, len);
        return int(HEC_OK);
    });
}

int hec_gf_matmul_device(hec_coder_t* c, const uint8_t* matrix, size_t rows, size_t cols,
                         const uint8_t* const* d_in, const size_t* in_strides, uint8_t* const* d_out,
                         const size_t* out_strides, size_t cell_len, size_t stripes, void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_gf_matmul_device");
    if (!c) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        return matmul_batch(c->device, matrix, rows, cols, d_in, in_strides, d_out, out_strides, cell_len, stripes,
                            static_cast<hipStream_t>(hip_stream));
    });
}

int hec_encode_device(hec_coder_t* c, const uint8_t* const* d_data, const size_t* data_strides,
                      uint8_t* const* d_parity, const size_t* parity_strides, size_t cell_len, size_t stripes,
                      void* hip_stream) {
    if (!c) return HEC_ERR_INVALID_ARG;
    return hec_gf_matmul_device(c, c->enc.data() + c->k * c->k, c->m, c->k, d_data, data_strides, d_parity,
                                parity_strides, cell_len, stripes, hip_stream);
}

int hec_decode_device(hec_coder_t* c, const uint8_t* const* d_shards, const size_t* shard_strides,
                      uint8_t* const* d_out, const size_t* out_strides, size_t cell_len, size_t stripes,
                      void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_decode_device");
    if (!c || !d_shards || !shard_strides || cell_len == 0) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        uint8_t present[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < c->k + c->m; i++) present[i] = d_shards[i] != nullptr;
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;
        if (p.missing.empty()) return HEC_OK;
        if (!d_out || !out_strides) return HEC_ERR_INVALID_ARG;
        const uint8_t* in[HEC_MAX_DATA_UNITS];
        size_t ist[HEC_MAX_DATA_UNITS];
        uint8_t* out[HEC_MAX_DATA_UNITS];
        size_t ost[HEC_MAX_DATA_UNITS];
        for (size_t r = 0; r < c->k; r++) {
            in[r] = d_shards[p.survivors[r]];
            ist[r] = shard_strides[p.survivors[r]];
        }
        for (size_t r = 0; r < p.missing.size(); r++) {
            out[r] = d_out[p.missing[r]];
            ost[r] = out_strides[p.missing[r]];
        }
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        return matmul_batch(c->device, p.matrix.data(), p.missing.size(), c->k, in, ist, out, ost, cell_len, stripes,
                            static_cast<hipStream_t>(hip_stream));
    });
}

int hec_encode(hec_coder_t* c, const uint8_t* const* data, size_t shard_len, uint8_t* const* parity) {
    if (!c || !data || !parity || shard_len == 0) return HEC_ERR_INVALID_ARG;
    for (size_t i = 0; i < c->k; i++)
        if (!data[i]) return HEC_ERR_INVALID_ARG;
    for (size_t j = 0; j < c->m; j++)
        if (!parity[j]) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        // small rows are coded on this thread (no PCIe round trip, no lock)
        return code_row(c, c->enc.data() + c->k * c->k, c->enc_aff.data(), data, c->k, parity, c->m, shard_len);
    });
}

int hec_decode(hec_coder_t* c, const uint8_t* const* shards, size_t shard_len, uint8_t* const* out) {
    if (!c || !shards || shard_len == 0) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        uint8_t present[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < c->k + c->m; i++) present[i] = shards[i] != nullptr;
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;
        if (p.missing.empty()) return HEC_OK;
        if (!out) return HEC_ERR_INVALID_ARG;
        for (size_t i : p.missing)
            if (!out[i]) return HEC_ERR_INVALID_ARG;
        const uint8_t* in[HEC_MAX_DATA_UNITS];
        uint8_t* dst[HEC_MAX_DATA_UNITS];
        for (size_t r = 0; r < c->k; r++) in[r] = shards[p.survivors[r]];
        for (size_t r = 0; r < p.missing.size(); r++) dst[r] = out[p.missing[r]];
        return code_row(c, p.matrix.data(), p.aff.data(), in, c->k, dst, p.missing.size(), shard_len);
    });
}

// ---- heterogeneous per-stripe erasure patterns ---------------------------

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }

size_t max_plans(size_t k, size_t m, size_t stripes) {
    // presence masks with >= 1 missing data shard and >= k present: at most
    // sum_{j=1..m} C(k+m, j)
    double total = 0, c = 1;
    for (size_t j = 1; j <= m; j++) {
        c = c * double(k + m - j + 1) / double(j);
        total += c;
    }
    return std::min(stripes, size_t(total));
}

size_t plan_bytes(size_t k, size_t m) {
    return sizeof(hec::DevPlanHeader) + std::min(k, m) * k * sizeof(hec::PermTable);
}

// [per-stripe plan offset: u32 x stripes][plan blob][launch tile counters]
// (hec::MixedArgs)
size_t mixed_workspace(size_t k, size_t m, size_t stripes) {
    const size_t p = max_plans(k, m, stripes);
    return align_up(align_up(stripes * sizeof(uint32_t)) + p * plan_bytes(k, m)) + hec::kMixedQueueBytes;
}


}  // namespace

size_t hec_decode_mixed_workspace_size(const hec_coder_t* c, size_t stripes) {
    if (!c) return 0;
    return mixed_workspace(c->k, c->m, stripes);
}

namespace {

// Body of hec_decode_device_mixed.  Shards that no stripe's plan reads may be
// null here (the verified read's phase 2); the public call requires storage
// for every shard index.
int mixed_decode_impl(hec_coder* c, const uint8_t* const* d_shards, const size_t* shard_strides,
                      uint8_t* const* d_out, const size_t* out_strides, const uint64_t* present, size_t cell_len,
                      size_t stripes, void* d_workspace, size_t workspace_bytes, void* hip_stream) {
    {
        const size_t k = c->k, m = c->m, n = k + m;
        const uint64_t all = n >= 64 ? ~uint64_t(0) : ((uint64_t(1) << n) - 1);
        // 1. plan per distinct mask (host), fail before launching anything
        std::map<uint64_t, uint16_t> ids;
        std::vector<PlanRef> plans;
        std::vector<uint16_t> stripe_plan(stripes);
        size_t max_e = 0;
        for (size_t s = 0; s < stripes; s++) {
            const uint64_t mask = present[s] & all;
            auto it = ids.find(mask);
            if (it == ids.end()) {
                uint8_t pres[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
                for (size_t i = 0; i < n; i++) pres[i] = (mask >> i) & 1;
                const PlanRef p_ref = cached_plan(c, pres);
                const DecodePlan& p = *p_ref;
                if (p.status != HEC_OK) return p.status;
                uint16_t id = 0xFFFF;
                if (!p.missing.empty()) {
                    if (plans.size() >= 0xFFFF) return HEC_ERR_INVALID_ARG;
                    id = uint16_t(plans.size());
                    plans.push_back(p_ref);
                    max_e = std::max(max_e, p.missing.size());
                }
                it = ids.emplace(mask, id).first;
            }
            stripe_plan[s] = it->second;
        }
        if (plans.empty()) return HEC_OK;
        for (const PlanRef& p : plans)
            for (size_t i : p->missing)
                if (!d_out[i]) return HEC_ERR_INVALID_ARG;
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        hipStream_t stream = static_cast<hipStream_t>(hip_stream);

        bool aligned = cell_len % 16 == 0;
        for (size_t i = 0; i < n; i++)
            aligned &= ((reinterpret_cast<uintptr_t>(d_shards[i]) | shard_strides[i]) & 15u) == 0;
        for (size_t i = 0; i < k; i++)
            aligned &= ((reinterpret_cast<uintptr_t>(d_out[i]) | out_strides[i]) & 15u) == 0;
        const bool fused = aligned && (k == 2 || k == 3 || k == 6 || k == 10);

        if (!fused) {
            // Correct for any shape: one uniform-pattern launch per run of
            // consecutive stripes sharing a plan.
            size_t s0 = 0;
            while (s0 < stripes) {
                size_t s1 = s0 + 1;
                while (s1 < stripes && stripe_plan[s1] == stripe_plan[s0]) s1++;
                if (stripe_plan[s0] != 0xFFFF) {
                    const DecodePlan& p = *plans[stripe_plan[s0]];
                    const uint8_t* in[HEC_MAX_DATA_UNITS];
                    size_t ist[HEC_MAX_DATA_UNITS];
                    uint8_t* out[HEC_MAX_DATA_UNITS];
                    size_t ost[HEC_MAX_DATA_UNITS];
                    for (size_t r = 0; r < k; r++) {
                        in[r] = d_shards[p.survivors[r]] + s0 * shard_strides[p.survivors[r]];
                        ist[r] = shard_strides[p.survivors[r]];
                    }
                    for (size_t r = 0; r < p.missing.size(); r++) {
                        out[r] = d_out[p.missing[r]] + s0 * out_strides[p.missing[r]];
                        ost[r] = out_strides[p.missing[r]];
                    }
                    const int rc = matmul_batch(c->device, p.matrix.data(), p.missing.size(), k, in, ist, out, ost,
                                                cell_len, s1 - s0, stream);
                    if (rc != HEC_OK) return rc;
                }
                s0 = s1;
            }
            return HEC_OK;
        }

        // 2. workspace image: per-stripe plan offsets | plan blobs
        const size_t blob_pos = align_up(stripes * sizeof(uint32_t));
        size_t blob_bytes = 0;
        std::vector<uint32_t> plan_off(plans.size());
        for (size_t pi = 0; pi < plans.size(); pi++) {
            plan_off[pi] = uint32_t(blob_bytes);
            blob_bytes += sizeof(hec::DevPlanHeader) + plans[pi]->missing.size() * k * sizeof(hec::PermTable);
        }
        const size_t queue_pos = align_up(blob_pos + blob_bytes);
        const size_t need = queue_pos + hec::kMixedQueueBytes;
        if (!d_workspace || workspace_bytes < need || blob_bytes > 0xFFFFFFF0ull) return HEC_ERR_INVALID_ARG;
        {
            // one of the coder's two pinned images, free once its last copy has run
            std::lock_guard<std::mutex> lk(c->mixed_mu);
            const int b = c->mixed_next;
            c->mixed_next ^= 1;
            if (!c->ev_mixed[b]) HEC_HIP(hipEventCreateWithFlags(&c->ev_mixed[b], hipEventDisableTiming), HEC_ERR_DEVICE);
            else HEC_HIP(hipEventSynchronize(c->ev_mixed[b]), HEC_ERR_DEVICE);
            if (c->mixed_host_bytes[b] < need) {
                if (c->mixed_host[b]) (void)hipHostFree(c->mixed_host[b]);
                c->mixed_host[b] = nullptr;
                c->mixed_host_bytes[b] = 0;
                const size_t want = std::max(need, 2 * c->mixed_host_bytes[b ^ 1]);
                HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->mixed_host[b]), want, hipHostMallocDefault),
                        HEC_ERR_NO_MEMORY);
                c->mixed_host_bytes[b] = want;
            }
            uint8_t* host = c->mixed_host[b];
            uint32_t* soff = reinterpret_cast<uint32_t*>(host);
            for (size_t s_ = 0; s_ < stripes; s_++)
                soff[s_] = stripe_plan[s_] == 0xFFFF ? hec::kNoPlan : plan_off[stripe_plan[s_]];
            for (size_t pi = 0; pi < plans.size(); pi++) {
                const DecodePlan& p = *plans[pi];
                auto* hdr = reinterpret_cast<hec::DevPlanHeader*>(host + blob_pos + plan_off[pi]);
                std::memset(hdr, 0, sizeof(*hdr));
                hdr->e = uint32_t(p.missing.size());
                for (size_t r = 0; r < k; r++) hdr->surv[r] = uint8_t(p.survivors[r]);
                for (size_t r = 0; r < p.missing.size(); r++) hdr->miss[r] = uint8_t(p.missing[r]);
                std::memcpy(host + blob_pos + plan_off[pi] + sizeof(hec::DevPlanHeader), p.perm.data(),
                            p.perm.size() * sizeof(uint32_t));
            }
            std::memset(host + blob_pos + blob_bytes, 0, need - (blob_pos + blob_bytes));  // pad + zeroed counters
            HEC_HIP(hipMemcpyAsync(d_workspace, host, need, hipMemcpyHostToDevice, stream), HEC_ERR_DEVICE);
            HEC_HIP(hipEventRecord(c->ev_mixed[b], stream), HEC_ERR_DEVICE);
        }

        // 3. one launch per group of <= 4 missing rows
        hec::MixedArgs a;
        std::memset(&a, 0, sizeof(a));
        for (size_t i = 0; i < n; i++) {
            a.base[i] = d_shards[i];
            a.stride[i] = shard_strides[i];
        }
        for (size_t i = 0; i < k; i++) {
            a.out[i] = d_out[i];
            a.out_stride[i] = out_strides[i];
        }
        uint8_t* ws = static_cast<uint8_t*>(d_workspace);
        a.stripe_off = reinterpret_cast<const uint32_t*>(ws);
        a.plans = ws + blob_pos;
        a.blob_bytes = uint32_t(blob_bytes);
        a.k = int32_t(k);
        a.cell_len = cell_len;
        a.stripes = stripes;
        for (size_t r0 = 0; r0 < max_e; r0 += hec::kMaxR) {
            a.row0 = int32_t(r0);
            a.queue = reinterpret_cast<uint32_t*>(ws + queue_pos + (r0 / hec::kMaxR) * hec::kMixedQueues *
                                                                          hec::kMixedQueueStride);
            const int rows = int(std::min(max_e - r0, size_t(hec::kMaxR)));
            const int rc = hec::launch_decode_mixed(a, rows, c->device, stream);
            if (rc != 0) return to_status(rc);
        }
        return HEC_OK;
    }
}

}  // namespace

int hec_decode_device_mixed(hec_coder_t* c, const uint8_t* const* d_shards, const size_t* shard_strides,
                            uint8_t* const* d_out, const size_t* out_strides, const uint64_t* present,
                            size_t cell_len, size_t stripes, void* d_workspace, size_t workspace_bytes,
                            void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_decode_device_mixed");
    if (!c || !d_shards || !shard_strides || !d_out || !out_strides || !present || cell_len == 0)
        return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    if (stripes > 0xFFFFFFFFull) return HEC_ERR_INVALID_ARG;
    for (size_t i = 0; i < c->k + c->m; i++)
        if (!d_shards[i]) return HEC_ERR_INVALID_ARG;  // every shard needs storage (present in some stripe)
    return guarded([&] {
        return mixed_decode_impl(c, d_shards, shard_strides, d_out, out_strides, present, cell_len, stripes,
                                 d_workspace, workspace_bytes, hip_stream);
    });
}

// Pipelined pinned-host batch, 3 device slots and 3 streams:
//   h2d stream:     [wait kernel(q-3) done: input slot free] H2D(q)  -> ev_in[slot]
//   compute stream: [wait ev_in[slot], D2H(q-3) done: output slot free] encode(q) -> ev_k[slot]
//   d2h stream:     [wait ev_k[slot]] D2H(q) -> ev_out[slot]
// so chunk q+1's H2D, chunk q's encode and chunk q-1's D2H run concurrently
// (PCIe is full duplex; the SDMA engines serve both directions at once).
int hec_encode_host_batch(hec_coder_t* c, const uint8_t* h_data, uint8_t* h_parity, size_t cell_len,
                          size_t stripes, size_t chunk_stripes) {
    if (!c || !h_data || !h_parity || cell_len == 0 || chunk_stripes == 0) return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    if (c->device == HEC_DEVICE_HOST) {  // host-only coder: the host routine, stripe by stripe
        return guarded([&] {
            const size_t k = c->k, m = c->m;
            const uint8_t* in[HEC_MAX_DATA_UNITS];
            uint8_t* out[HEC_MAX_PARITY_UNITS];
            for (size_t s = 0; s < stripes; s++) {
                for (size_t i = 0; i < k; i++) in[i] = h_data + (s * k + i) * cell_len;
                for (size_t j = 0; j < m; j++) out[j] = h_parity + (s * m + j) * cell_len;
                hec::host::gf_matmul_split(c->enc.data() + k * k, c->enc_aff.data(), m, k, in, out, cell_len);
            }
            return int(HEC_OK);
        });
    }
    return guarded([&] {
        std::lock_guard<std::mutex> lk(c->host_mu);
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        StreamDrain drain{c};
        const size_t k = c->k, m = c->m;
        constexpr int kSlots = hec_coder::kSlots;
        chunk_stripes = std::min(chunk_stripes, stripes);
        const size_t in_bytes = chunk_stripes * k * cell_len;
        const size_t out_bytes = chunk_stripes * m * cell_len;
        const size_t slot_bytes = in_bytes + out_bytes;
        int rc = ensure_dbuf(c, kSlots * slot_bytes);
        if (rc != HEC_OK) return rc;
        hipStream_t h2d = c->copy_stream[0], d2h = c->copy_stream[1];
        const size_t nchunks = (stripes + chunk_stripes - 1) / chunk_stripes;
        for (size_t q = 0; q < nchunks; q++) {
            const int slot = int(q % kSlots);
            uint8_t* din = c->dbuf + slot * slot_bytes;
            uint8_t* dpar = din + in_bytes;
            const size_t s0 = q * chunk_stripes;
            const size_t ns = std::min(chunk_stripes, stripes - s0);
            if (q >= size_t(kSlots)) HEC_HIP(hipStreamWaitEvent(h2d, c->ev_k[slot], 0), HEC_ERR_DEVICE);
            HEC_HIP(hipMemcpyAsync(din, h_data + s0 * k * cell_len, ns * k * cell_len, hipMemcpyHostToDevice, h2d),
                    HEC_ERR_DEVICE);
            HEC_HIP(hipEventRecord(c->ev_in[slot], h2d), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamWaitEvent(c->stream, c->ev_in[slot], 0), HEC_ERR_DEVICE);
            if (q >= size_t(kSlots)) HEC_HIP(hipStreamWaitEvent(c->stream, c->ev_out[slot], 0), HEC_ERR_DEVICE);
            const uint8_t* in[HEC_MAX_DATA_UNITS];
            uint8_t* out[HEC_MAX_PARITY_UNITS];
            size_t ist[HEC_MAX_DATA_UNITS], ost[HEC_MAX_PARITY_UNITS];
            for (size_t i = 0; i < k; i++) {
                in[i] = din + i * cell_len;
                ist[i] = k * cell_len;
            }
            for (size_t j = 0; j < m; j++) {
                out[j] = dpar + j * cell_len;
                ost[j] = m * cell_len;
            }
            rc = matmul_batch(c->device, c->enc.data() + k * k, m, k, in, ist, out, ost, cell_len, ns, c->stream);
            if (rc != HEC_OK) return rc;
            HEC_HIP(hipEventRecord(c->ev_k[slot], c->stream), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamWaitEvent(d2h, c->ev_k[slot], 0), HEC_ERR_DEVICE);
            HEC_HIP(hipMemcpyAsync(h_parity + s0 * m * cell_len, dpar, ns * m * cell_len, hipMemcpyDeviceToHost, d2h),
                    HEC_ERR_DEVICE);
            HEC_HIP(hipEventRecord(c->ev_out[slot], d2h), HEC_ERR_DEVICE);
        }
        HEC_HIP(hipStreamSynchronize(h2d), HEC_ERR_DEVICE);
        HEC_HIP(hipStreamSynchronize(c->stream), HEC_ERR_DEVICE);
        HEC_HIP(hipStreamSynchronize(d2h), HEC_ERR_DEVICE);
        return HEC_OK;
    });
}

// Pipelined pinned-host decode straight into file order (the reader's
// ec_decode + cell split + concatenation, ec/mod.rs:62-89 and
// block_reader.rs:480-554, in one pass).  The k survivors go H2D, one
// contiguous copy per shard per chunk; the decode kernel writes the e missing
// cells to a compact region; only those come back D2H, each as a 2D copy into
// its file slots.  The present data
// cells never make the round trip: host threads copy them from the vertical
// buffers into their file slots while the DMA engines run, so PCIe carries
// k cells in and e cells out per row instead of k in and k out.
int hec_decode_host_batch(hec_coder_t* c, const uint8_t* const* h_vertical, size_t cell_len, size_t rows,
                          uint8_t* h_file, size_t chunk_rows) {
    if (!c || !h_vertical || !h_file || cell_len == 0 || chunk_rows == 0) return HEC_ERR_INVALID_ARG;
    if (rows == 0) return HEC_OK;
    return guarded([&] {
        const size_t k = c->k, m = c->m;
        uint8_t present[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < k + m; i++) present[i] = h_vertical[i] != nullptr;
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;

        // host side: present data cells -> file slots, rows split over up to
        // 4 threads (the caller's thread takes the first share)
        auto copy_rows = [&](size_t ra, size_t rb) {
            for (size_t r = ra; r < rb; r++)
                for (size_t i = 0; i < k; i++)
                    if (h_vertical[i])
                        std::memcpy(h_file + (r * k + i) * cell_len, h_vertical[i] + r * cell_len, cell_len);
        };
        const size_t copy_bytes = rows * (k - p.missing.size()) * cell_len;
        const int tuned_threads = hec::tune_snapshot().host_copy_threads;
        const size_t max_threads = tuned_threads > 0 ? size_t(tuned_threads) : 4;
        const size_t nthreads = std::min<size_t>(max_threads, std::max<size_t>(1, copy_bytes >> 24));  // >= 16 MiB each
        std::vector<std::thread> copiers;
        auto join_copiers = [&] {
            for (auto& t : copiers) t.join();
            copiers.clear();
        };
        size_t own_a = 0, own_b = rows;
        if (nthreads > 1) {
            copiers.reserve(nthreads - 1);
            for (size_t t = 1; t < nthreads; t++) {
                const size_t ra = rows * t / nthreads, rb = rows * (t + 1) / nthreads;
                try {
                    copiers.emplace_back(copy_rows, ra, rb);
                } catch (...) {
                    copy_rows(ra, rb);  // no thread: copy inline
                }
            }
            own_b = rows / nthreads;
        }
        if (p.missing.empty()) {  // nothing to rebuild: a pure host copy
            copy_rows(own_a, own_b);
            join_copiers();
            return HEC_OK;
        }

        int rc = [&]() -> int {
            if (c->device == HEC_DEVICE_HOST) {  // host-only coder: rebuild row by row on this thread
                const size_t e = p.missing.size();
                const uint8_t* in[HEC_MAX_DATA_UNITS];
                uint8_t* out[HEC_MAX_DATA_UNITS];
                for (size_t r = 0; r < rows; r++) {
                    for (size_t i = 0; i < k; i++) in[i] = h_vertical[p.survivors[i]] + r * cell_len;
                    for (size_t i = 0; i < e; i++) out[i] = h_file + (r * k + p.missing[i]) * cell_len;
                    hec::host::gf_matmul_split(p.matrix.data(), p.aff.data(), e, k, in, out, cell_len);
                }
                copy_rows(own_a, own_b);
                return int(HEC_OK);
            }
            std::lock_guard<std::mutex> lk(c->host_mu);
            DeviceGuard g(c->device);
            if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
            StreamDrain drain{c};  // before join_copiers and before returning, also on errors
            constexpr int kSlots = hec_coder::kSlots;
            chunk_rows = std::min(chunk_rows, rows);
            // slot: the k survivors shard-major [k][chunk][cell] (one
            // contiguous H2D per survivor), then the e rebuilt cells
            // [e][chunk][cell] (one 2D D2H per missing shard into its file slots)
            const size_t e = p.missing.size();
            const size_t shard_bytes = chunk_rows * cell_len;
            const size_t slot_bytes = (k + e) * shard_bytes;
            int rc2 = ensure_dbuf(c, kSlots * slot_bytes);
            if (rc2 != HEC_OK) return rc2;
            hipStream_t h2d = c->copy_stream[0], d2h = c->copy_stream[1];
            const size_t nchunks = (rows + chunk_rows - 1) / chunk_rows;
            for (size_t q = 0; q < nchunks; q++) {
                const int slot = int(q % kSlots);
                uint8_t* dsurv = c->dbuf + slot * slot_bytes;
                uint8_t* dmiss = dsurv + k * shard_bytes;
                const size_t r0 = q * chunk_rows;
                const size_t nr = std::min(chunk_rows, rows - r0);
                // slot reuse: the D2H of chunk q-3 (which follows its kernel) is done
                if (q >= size_t(kSlots)) HEC_HIP(hipStreamWaitEvent(h2d, c->ev_out[slot], 0), HEC_ERR_DEVICE);
                for (size_t r = 0; r < k; r++)
                    HEC_HIP(hipMemcpyAsync(dsurv + r * shard_bytes, h_vertical[p.survivors[r]] + r0 * cell_len,
                                           nr * cell_len, hipMemcpyHostToDevice, h2d),
                            HEC_ERR_DEVICE);
                HEC_HIP(hipEventRecord(c->ev_in[slot], h2d), HEC_ERR_DEVICE);
                HEC_HIP(hipStreamWaitEvent(c->stream, c->ev_in[slot], 0), HEC_ERR_DEVICE);
                const uint8_t* in[HEC_MAX_DATA_UNITS];
                size_t ist[HEC_MAX_DATA_UNITS];
                uint8_t* out[HEC_MAX_DATA_UNITS];
                size_t ost[HEC_MAX_DATA_UNITS];
                for (size_t r = 0; r < k; r++) {
                    in[r] = dsurv + r * shard_bytes;
                    ist[r] = cell_len;
                }
                for (size_t r = 0; r < e; r++) {
                    out[r] = dmiss + r * shard_bytes;
                    ost[r] = cell_len;
                }
                rc2 = matmul_batch(c->device, p.matrix.data(), e, k, in, ist, out, ost, cell_len, nr, c->stream);
                if (rc2 != HEC_OK) return rc2;
                HEC_HIP(hipEventRecord(c->ev_k[slot], c->stream), HEC_ERR_DEVICE);
                HEC_HIP(hipStreamWaitEvent(d2h, c->ev_k[slot], 0), HEC_ERR_DEVICE);
                for (size_t r = 0; r < e; r++)  // rebuilt cells only, into their file slots
                    HEC_HIP(hipMemcpy2DAsync(h_file + (r0 * k + p.missing[r]) * cell_len, k * cell_len,
                                             dmiss + r * shard_bytes, cell_len, cell_len, nr, hipMemcpyDeviceToHost,
                                             d2h),
                            HEC_ERR_DEVICE);
                HEC_HIP(hipEventRecord(c->ev_out[slot], d2h), HEC_ERR_DEVICE);
            }
            // every chunk is enqueued (the waits are device-side): the caller's
            // host share runs while the DMA engines and the kernel work
            copy_rows(own_a, own_b);
            HEC_HIP(hipStreamSynchronize(h2d), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamSynchronize(c->stream), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamSynchronize(d2h), HEC_ERR_DEVICE);
            return HEC_OK;
        }();
        join_copiers();  // always, also on a device error (never leave a joinable thread)
        return rc;
    });
}

// ---- whole files: rows of k cells, the last one possibly short ---------------
// CellBuffer (block_writer.rs:791-851) fills cell 0 of a row before cell 1,
// so the last row of a file of data_len bytes holds L = data_len - full*k*cell
// bytes: cell i has min(cell, max(0, L - i*cell)) of them, and encode pads
// every cell with zeros to len(cell 0) = n0 = min(cell, L) and emits parity
// cells of n0 bytes.  The reader pads every short or absent cell with zeros
// to cell_size (CellReader::next_cell, block_reader.rs:343-378) before
// ec_decode, then trims the row to the file length (:524-549).

size_t hec_encode_rows_workspace_size(const hec_coder_t* c, size_t cell_len) {
    if (!c) return 0;
    return c->k * cell_len;  // the last row's short data cells, zero-padded
}

int hec_encode_rows_host(hec_coder_t* c, const uint8_t* h_data, size_t data_len, uint8_t* h_parity, size_t cell_len,
                         size_t chunk_stripes) {
    if (!c || !h_data || !h_parity || cell_len == 0 || chunk_stripes == 0) return HEC_ERR_INVALID_ARG;
    if (data_len == 0) return HEC_OK;
    const size_t k = c->k, m = c->m, row = k * cell_len;
    const size_t full = data_len / row, L = data_len - full * row;
    if (full) {
        const int rc = hec_encode_host_batch(c, h_data, h_parity, cell_len, full, chunk_stripes);
        if (rc != HEC_OK || L == 0) return rc;
    }
    return guarded([&] {
        // the short last row: cells padded to n0 on the host, one row coded
        const size_t n0 = std::min(cell_len, L);
        const uint8_t* base = h_data + full * row;
        std::vector<uint8_t> pad(k * n0, 0);
        const uint8_t* in[HEC_MAX_DATA_UNITS];
        uint8_t* out[HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < k; i++) {
            const size_t have = L > i * cell_len ? std::min(cell_len, L - i * cell_len) : 0;
            if (have == n0) {
                in[i] = base + i * cell_len;  // a full-length cell is read in place
            } else {
                std::memcpy(&pad[i * n0], base + i * cell_len, have);
                in[i] = &pad[i * n0];
            }
        }
        uint8_t* pbase = h_parity + full * m * cell_len;
        for (size_t j = 0; j < m; j++) {
            out[j] = pbase + j * cell_len;
            std::memset(out[j] + n0, 0, cell_len - n0);  // the parity cell holds n0 bytes
        }
        return code_row(c, c->enc.data() + k * k, c->enc_aff.data(), in, k, out, m, n0);
    });
}

int hec_encode_rows_device(hec_coder_t* c, const uint8_t* d_data, size_t data_len, uint8_t* d_parity, size_t cell_len,
                           void* d_workspace, size_t workspace_bytes, void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_encode_rows_device");
    if (!c || !d_data || !d_parity || cell_len == 0) return HEC_ERR_INVALID_ARG;
    if (data_len == 0) return HEC_OK;
    const size_t k = c->k, m = c->m, row = k * cell_len;
    const size_t full = data_len / row, L = data_len - full * row;
    const uint8_t* din[HEC_MAX_DATA_UNITS];
    uint8_t* dout[HEC_MAX_PARITY_UNITS];
    size_t ist[HEC_MAX_DATA_UNITS], ost[HEC_MAX_PARITY_UNITS];
    for (size_t i = 0; i < k; i++) {
        din[i] = d_data + i * cell_len;
        ist[i] = row;
    }
    for (size_t j = 0; j < m; j++) {
        dout[j] = d_parity + j * cell_len;
        ost[j] = m * cell_len;
    }
    // validate the workspace before anything is queued: a bad argument must not
    // leave the full rows' parity written and the short row's not.  It is
    // needed only when some cell of the short last row holds fewer than
    // n0 = min(cell, L) bytes (the zero-padded copies); k == 1, or a short
    // row whose cells all reach n0, needs none.
    const size_t n0 = std::min(cell_len, L);
    bool pad = false;
    for (size_t i = 0; i < k && L; i++) pad |= (L > i * cell_len ? std::min(cell_len, L - i * cell_len) : 0) < n0;
    if (pad && (!d_workspace || workspace_bytes < k * n0)) return HEC_ERR_INVALID_ARG;
    if (full) {
        const int rc = hec_encode_device(c, din, ist, dout, ost, cell_len, full, hip_stream);
        if (rc != HEC_OK || L == 0) return rc;
    }
    return guarded([&] {
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        hipStream_t stream = static_cast<hipStream_t>(hip_stream);
        const uint8_t* base = d_data + full * row;
        uint8_t* ws = static_cast<uint8_t*>(d_workspace);
        for (size_t i = 0; i < k; i++) {
            const size_t have = L > i * cell_len ? std::min(cell_len, L - i * cell_len) : 0;
            din[i] = base + i * cell_len;
            if (have < n0) {  // short or empty cell: zero-padded copy (never read past the data)
                uint8_t* p = ws + i * n0;
                if (have)
                    HEC_HIP(hipMemcpyAsync(p, base + i * cell_len, have, hipMemcpyDeviceToDevice, stream),
                            HEC_ERR_DEVICE);
                HEC_HIP(hipMemsetAsync(p + have, 0, n0 - have, stream), HEC_ERR_DEVICE);
                din[i] = p;
            }
        }
        for (size_t j = 0; j < m; j++) {
            dout[j] = d_parity + full * m * cell_len + j * cell_len;
            if (n0 < cell_len) HEC_HIP(hipMemsetAsync(dout[j] + n0, 0, cell_len - n0, stream), HEC_ERR_DEVICE);
        }
        return matmul_batch(c->device, c->enc.data() + k * k, m, k, din, ist, dout, ost, n0, 1, stream);
    });
}

int hec_decode_rows_host(hec_coder_t* c, const uint8_t* const* h_vertical, const size_t* vertical_len,
                         size_t cell_len, uint8_t* h_file, size_t file_len, size_t chunk_rows) {
    if (!c || !h_vertical || !vertical_len || !h_file || cell_len == 0 || chunk_rows == 0) return HEC_ERR_INVALID_ARG;
    if (file_len == 0) return HEC_OK;
    const size_t k = c->k, m = c->m, row = k * cell_len;
    const size_t full = file_len / row, L = file_len - full * row;
    // full rows: every present shard holds full * cell_len bytes (max_offset)
    for (size_t i = 0; i < k + m; i++)
        if (h_vertical[i] && vertical_len[i] < full * cell_len) return HEC_ERR_INVALID_ARG;
    if (full) {
        const int rc = hec_decode_host_batch(c, h_vertical, cell_len, full, h_file, chunk_rows);
        if (rc != HEC_OK || L == 0) return rc;
    }
    return guarded([&] {
        // the short last row: each present cell zero-padded (CellReader), only
        // the first n0 = min(cell, L) bytes carry data (every data cell of the
        // row is zero past n0, so are the parity cells)
        const size_t n0 = std::min(cell_len, L);
        uint8_t present[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < k + m; i++) present[i] = h_vertical[i] != nullptr;
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;
        uint8_t* frow = h_file + full * row;
        auto cell_have = [&](size_t i) {  // bytes of cell i of the row inside the file
            return L > i * cell_len ? std::min(cell_len, L - i * cell_len) : size_t(0);
        };
        for (size_t i = 0; i < k; i++) {  // present data cells: copied, zero-padded
            if (!h_vertical[i]) continue;
            const size_t want = cell_have(i);
            const size_t avail = vertical_len[i] > full * cell_len ? vertical_len[i] - full * cell_len : 0;
            const size_t cp = std::min(want, avail);
            std::memcpy(frow + i * cell_len, h_vertical[i] + full * cell_len, cp);
            std::memset(frow + i * cell_len + cp, 0, want - cp);
        }
        if (p.missing.empty()) return int(HEC_OK);
        std::vector<uint8_t> surv(k * n0, 0), rec(p.missing.size() * n0);
        const uint8_t* in[HEC_MAX_DATA_UNITS];
        uint8_t* out[HEC_MAX_DATA_UNITS];
        for (size_t r = 0; r < k; r++) {
            const size_t s = p.survivors[r];
            const size_t avail = vertical_len[s] > full * cell_len ? vertical_len[s] - full * cell_len : 0;
            std::memcpy(&surv[r * n0], h_vertical[s] + full * cell_len, std::min(avail, n0));
            in[r] = &surv[r * n0];
        }
        for (size_t r = 0; r < p.missing.size(); r++) out[r] = &rec[r * n0];
        const int rc = code_row(c, p.matrix.data(), p.aff.data(), in, k, out, p.missing.size(), n0);
        if (rc != HEC_OK) return rc;
        for (size_t r = 0; r < p.missing.size(); r++) {
            const size_t i = p.missing[r];
            std::memcpy(frow + i * cell_len, &rec[r * n0], cell_have(i));
        }
        return int(HEC_OK);
    });
}

// ---- Chunk checksums ------------------------------------

namespace {

// HEC_CHECKSUM_* (ChecksumTypeProto) -> crc::Kind; -1 for NULL / invalid
int crc_kind(int checksum_type) {
    switch (checksum_type) {
        case HEC_CHECKSUM_CRC32C: return hec::crc::kCrc32c;
        case HEC_CHECKSUM_CRC32: return hec::crc::kCksum;
        default: return -1;
    }
}

// One checksum launch over n_shards cells per stripe; cell (s, i) sits at
// s * n_total + sid[i] in the sums/flags layouts (sid == nullptr: identity).
int checksum_launch(hec_coder* c, int kind, const uint8_t* const* bases, const size_t* strides, const uint8_t* sid,
                    size_t n_shards, size_t n_total, size_t cell_len, size_t stripes, size_t bpc, uint8_t* out,
                    const uint8_t* expected, uint8_t* bad, hipStream_t stream,
                    const uint32_t* stripe_list = nullptr) {
    hec::CrcArgs a;
    std::memset(&a, 0, sizeof(a));
    a.stripe_list = stripe_list;
    for (size_t i = 0; i < n_shards; i++) {
        if (!bases[i]) return HEC_ERR_INVALID_ARG;
        a.base[i] = bases[i];
        a.stride[i] = strides[i];
        a.sid[i] = uint8_t(sid ? sid[i] : i);
    }
    a.n_total = uint32_t(n_total);
    a.out = out;
    a.expected = expected;
    a.bad = bad;
    a.kind = kind;
    a.n_shards = uint32_t(n_shards);
    a.cell_len = cell_len;
    a.stripes = stripes;
    a.bytes_per_checksum = bpc;
    const int rc = hec::launch_checksum(a, c->device, stream);
    return rc == 0 ? HEC_OK : to_status(rc);
}

int checksum_entry(hec_coder* c, int checksum_type, const uint8_t* const* d_bases, const size_t* strides,
                   size_t n_shards, size_t cell_len, size_t stripes, size_t bpc, uint8_t* d_out,
                   const uint8_t* d_expected, uint8_t* d_bad, void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("checksum_entry");
    const int kind = crc_kind(checksum_type);
    if (!c || !d_bases || !strides || kind < 0 || n_shards == 0 || n_shards > size_t(hec::kCrcMaxShards) ||
        cell_len == 0 || bpc == 0 || (!d_out && !d_expected) || (d_expected && !d_bad))
        return HEC_ERR_INVALID_ARG;
    for (size_t i = 0; i < n_shards; i++)
        if (!d_bases[i]) return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    return guarded([&] {
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        return checksum_launch(c, kind, d_bases, strides, nullptr, n_shards, n_shards, cell_len, stripes, bpc, d_out,
                               d_expected, d_bad, static_cast<hipStream_t>(hip_stream));
    });
}

}  // namespace

int hec_crc32c_device(hec_coder_t* c, const uint8_t* const* d_bases, const size_t* strides, size_t n_shards,
                      size_t cell_len, size_t stripes, size_t bytes_per_checksum, uint8_t* d_out, void* hip_stream) {
    if (!d_out) return HEC_ERR_INVALID_ARG;
    return checksum_entry(c, HEC_CHECKSUM_CRC32C, d_bases, strides, n_shards, cell_len, stripes, bytes_per_checksum,
                          d_out, nullptr, nullptr, hip_stream);
}

int hec_checksum_device(hec_coder_t* c, int checksum_type, const uint8_t* const* d_bases, const size_t* strides,
                        size_t n_shards, size_t cell_len, size_t stripes, size_t bytes_per_checksum, uint8_t* d_out,
                        void* hip_stream) {
    if (!d_out) return HEC_ERR_INVALID_ARG;
    return checksum_entry(c, checksum_type, d_bases, strides, n_shards, cell_len, stripes, bytes_per_checksum, d_out,
                          nullptr, nullptr, hip_stream);
}

int hec_checksum_verify_device(hec_coder_t* c, int checksum_type, const uint8_t* const* d_bases,
                               const size_t* strides, size_t n_shards, size_t cell_len, size_t stripes,
                               size_t bytes_per_checksum, const uint8_t* d_expected, uint8_t* d_bad,
                               void* hip_stream) {
    if (checksum_type == HEC_CHECKSUM_NULL) return c ? HEC_OK : HEC_ERR_INVALID_ARG;
    if (!d_expected || !d_bad) return HEC_ERR_INVALID_ARG;
    return checksum_entry(c, checksum_type, d_bases, strides, n_shards, cell_len, stripes, bytes_per_checksum,
                          nullptr, d_expected, d_bad, hip_stream);
}

int hec_encode_crc_device(hec_coder_t* c, const uint8_t* const* d_data, const size_t* data_strides,
                          uint8_t* const* d_parity, const size_t* parity_strides, size_t cell_len, size_t stripes,
                          size_t bytes_per_checksum, uint8_t* d_sums, void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_encode_crc_device");
    if (!c || !d_data || !data_strides || !d_parity || !parity_strides || !d_sums || cell_len == 0 ||
        bytes_per_checksum == 0)
        return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    // Fused single pass when the shape allows it (k in {2,3,6,10}, m <= 4,
    // 512-B chunks, 16-B aligned cells); otherwise encode, then checksum.
    if (bytes_per_checksum == 512 && c->m <= size_t(hec::kMaxR) && !hec::tune_snapshot().crc_unfused) {
        const int rc = guarded([&] {
            DeviceGuard g(c->device);
            if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
            hec::MatmulArgs a;
            std::memset(&a, 0, sizeof(a));
            for (size_t i = 0; i < c->k; i++) {
                if (!d_data[i]) return int(HEC_ERR_INVALID_ARG);
                a.in[i] = d_data[i];
                a.in_stride[i] = data_strides[i];
            }
            for (size_t j = 0; j < c->m; j++) {
                if (!d_parity[j]) return int(HEC_ERR_INVALID_ARG);
                a.out[j] = d_parity[j];
                a.out_stride[j] = parity_strides[j];
                for (size_t i = 0; i < c->k; i++) a.coef[j * hec::kMaxK + i] = c->enc[(c->k + j) * c->k + i];
            }
            a.k = int32_t(c->k);
            a.r = int32_t(c->m);
            a.cell_len = cell_len;
            a.stripes = stripes;
            hec::FusedCrcArgs cs;
            std::memset(&cs, 0, sizeof(cs));
            cs.sums = d_sums;
            cs.n_total = uint32_t(c->k + c->m);
            cs.kind = hec::crc::kCrc32c;
            for (size_t i = 0; i < c->k + c->m; i++) cs.shard_id[i] = uint8_t(i);
            const int lrc = hec::launch_encode_crc(a, cs, c->device, static_cast<hipStream_t>(hip_stream));
            if (lrc == -1) return 1;  // shape not covered: fall through
            return lrc == 0 ? int(HEC_OK) : to_status(lrc);
        });
        if (rc != 1) return rc;
    }
    int rc = hec_encode_device(c, d_data, data_strides, d_parity, parity_strides, cell_len, stripes, hip_stream);
    if (rc != HEC_OK) return rc;
    const uint8_t* bases[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
    size_t st[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
    for (size_t i = 0; i < c->k; i++) {
        bases[i] = d_data[i];
        st[i] = data_strides[i];
    }
    for (size_t j = 0; j < c->m; j++) {
        bases[c->k + j] = d_parity[j];
        st[c->k + j] = parity_strides[j];
    }
    return hec_crc32c_device(c, bases, st, c->k + c->m, cell_len, stripes, bytes_per_checksum, d_sums, hip_stream);
}

// The verified striped read (block_reader.rs:480-525 -> ec_decode): phase 1
// verifies the batch plan's survivors of every stripe and rebuilds its
// missing data in one pass; phase 2 re-plans, one stripe at a time, the
// stripes where a survivor failed: drop it, take the next available shard
// (verifying it first, as read_slice starts the next parity reader), and
// rebuild every missing or failed data cell of that stripe.
// ---- plan-time specialisation of the fused decode + verify kernel (jit.hpp) ----

int hec_coder_prepare_decode(hec_coder_t* c, const uint8_t* present, int checksum_type, int* specialised) {
    if (specialised) *specialised = 0;
    if (!c || !present) return HEC_ERR_INVALID_ARG;
    const int kind = crc_kind(checksum_type);
    if (kind < 0) return HEC_ERR_INVALID_ARG;
    if (c->device == HEC_DEVICE_HOST) return host_only("hec_coder_prepare_decode");
    return guarded([&]() -> int {
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;
        if (p.missing.empty() || p.missing.size() > size_t(hec::kMaxR)) return int(HEC_OK);  // no fused decode
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        hec::jit::VerifyKernel vk;
        const int e = int(p.missing.size());
        const hec::Tune tn = hec::tune_snapshot();
        const int slabs = (tn.fused_slabs == 4 || tn.fused_slabs == 8) ? tn.fused_slabs
                                                                        : hec::jit::default_slabs(int(c->k), e);
        const int pfd = hec::jit::pick_pfd(tn.jit_pfd, slabs, int(c->k), e);
        const int wpe = tn.fused_wpe == 3 && slabs == 4 ? 3 : 2;
        const int scheme = tn.crc_variant == 12 && kind == 0 ? 15 : 12;  // measurement: slicing-by-32 tail
        // the launch's choice (ec_fused.hip launch_fused; measurement: tune key 28)
        const bool wq = (hec::kExperimental && tn.fused_wq) ? tn.fused_wq == 1 : hec::jit::default_wq(int(c->k), e);
        const bool ok = hec::jit::verify_kernel(c->device, int(c->k), e, kind, slabs, wpe, pfd, p.matrix.data(), true,
                                                &vk, scheme, wq);
        if (specialised) *specialised = ok ? 1 : 0;
        return int(HEC_OK);
    });
}

int hec_jit_warm(size_t data_units, size_t parity_units, const uint8_t* present, int checksum_type) {
    if (!present || data_units == 0 || data_units > HEC_MAX_DATA_UNITS || parity_units == 0 ||
        parity_units > HEC_MAX_PARITY_UNITS)
        return HEC_ERR_INVALID_ARG;
    const int kind = crc_kind(checksum_type);
    if (kind < 0) return HEC_ERR_INVALID_ARG;
    return guarded([&]() -> int {
        size_t e = 0, surv[HEC_MAX_DATA_UNITS], miss[HEC_MAX_DATA_UNITS];
        uint8_t mat[HEC_MAX_DATA_UNITS * HEC_MAX_DATA_UNITS];
        const int rc = hec_decode_plan(data_units, parity_units, present, &e, surv, miss, mat);
        if (rc != HEC_OK) return rc;
        const size_t k = data_units;
        if (e == 0 || e > size_t(hec::kMaxR) || !(k == 2 || k == 3 || k == 6 || k == 10)) return int(HEC_ERR_INVALID_ARG);
        return hec::jit::warm(int(k), int(e), kind, hec::jit::default_slabs(int(k), int(e)), 2,
                              hec::jit::default_pfd(int(k), int(e)), mat, 12,
                              hec::jit::default_wq(int(k), int(e))) ? int(HEC_OK)
                                                         : fail(HEC_ERR_DEVICE, "hiprtc compile", hipErrorNotSupported);
    });
}

void hec_jit_stats(uint64_t* compiled, uint64_t* from_disk, uint64_t* failed, uint64_t* launches) {
    const hec::jit::Stats st = hec::jit::stats();
    if (compiled) *compiled = st.compiled;
    if (from_disk) *from_disk = st.from_disk;
    if (failed) *failed = st.failed;
    if (launches) *launches = st.launches;
}

int hec_decode_verify_device(hec_coder_t* c, int checksum_type, const uint8_t* const* d_shards,
                             const size_t* shard_strides, uint8_t* const* d_out, const size_t* out_strides,
                             size_t cell_len, size_t stripes, size_t bytes_per_checksum, const uint8_t* d_sums,
                             uint8_t* d_bad, void* hip_stream) {
    if (c && c->device == HEC_DEVICE_HOST) return host_only("hec_decode_verify_device");
    if (!c || !d_shards || !shard_strides || !d_out || !out_strides || cell_len == 0) return HEC_ERR_INVALID_ARG;
    if (checksum_type == HEC_CHECKSUM_NULL)
        return hec_decode_device(c, d_shards, shard_strides, d_out, out_strides, cell_len, stripes, hip_stream);
    const int kind = crc_kind(checksum_type);
    if (kind < 0 || bytes_per_checksum == 0 || !d_sums || !d_bad) return HEC_ERR_INVALID_ARG;
    for (size_t i = 0; i < c->k; i++)
        if (!d_out[i]) return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    return guarded([&]() -> int {
        const size_t k = c->k, n = c->k + c->m;
        const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
        uint8_t present[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
        for (size_t i = 0; i < n; i++) present[i] = d_shards[i] != nullptr;
        const PlanRef p_ref = cached_plan(c, present);
        const DecodePlan& p = *p_ref;
        if (p.status != HEC_OK) return p.status;  // fewer than k available: nothing is read
        std::vector<size_t> surv = p.survivors;
        if (p.missing.empty())
            for (size_t i = 0; i < k; i++) surv.push_back(i);  // nothing to rebuild: the data cells are read
        DeviceGuard g(c->device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        HEC_HIP(hipMemsetAsync(d_bad, 0, stripes * n, stream), HEC_ERR_DEVICE);

        // ---- phase 1: the whole batch under the batch plan
        const uint8_t* in[HEC_MAX_DATA_UNITS];
        size_t ist[HEC_MAX_DATA_UNITS];
        uint8_t sid[HEC_MAX_DATA_UNITS];
        for (size_t r = 0; r < k; r++) {
            in[r] = d_shards[surv[r]];
            ist[r] = shard_strides[surv[r]];
            sid[r] = uint8_t(surv[r]);
        }
        bool fused = false;
        if (!p.missing.empty() && p.missing.size() <= size_t(hec::kMaxR) && bytes_per_checksum == 512) {
            hec::MatmulArgs a;
            std::memset(&a, 0, sizeof(a));
            for (size_t r = 0; r < k; r++) {
                a.in[r] = in[r];
                a.in_stride[r] = ist[r];
            }
            for (size_t j = 0; j < p.missing.size(); j++) {
                a.out[j] = d_out[p.missing[j]];
                a.out_stride[j] = out_strides[p.missing[j]];
                for (size_t i = 0; i < k; i++) a.coef[j * hec::kMaxK + i] = p.matrix[j * k + i];
            }
            a.k = int32_t(k);
            a.r = int32_t(p.missing.size());
            a.cell_len = cell_len;
            a.stripes = stripes;
            hec::FusedCrcArgs cs;
            std::memset(&cs, 0, sizeof(cs));
            cs.expected = d_sums;
            cs.bad = d_bad;
            cs.n_total = uint32_t(n);
            cs.kind = kind;
            for (size_t r = 0; r < k; r++) cs.shard_id[r] = sid[r];
            const int lrc = hec::launch_decode_verify(a, cs, c->device, stream);
            if (lrc > 0) return to_status(lrc);
            fused = lrc == 0;
        }
        if (!fused) {
            int rc = checksum_launch(c, kind, in, ist, sid, k, n, cell_len, stripes, bytes_per_checksum, nullptr,
                                     d_sums, d_bad, stream);
            if (rc != HEC_OK) return rc;
            if (!p.missing.empty()) {
                uint8_t* out[HEC_MAX_DATA_UNITS];
                size_t ost[HEC_MAX_DATA_UNITS];
                for (size_t j = 0; j < p.missing.size(); j++) {
                    out[j] = d_out[p.missing[j]];
                    ost[j] = out_strides[p.missing[j]];
                }
                rc = matmul_batch(c->device, p.matrix.data(), p.missing.size(), k, in, ist, out, ost, cell_len, stripes,
                                  stream);
                if (rc != HEC_OK) return rc;
            }
        }
        std::vector<uint8_t> bad(stripes * n);
        HEC_HIP(hipMemcpyAsync(bad.data(), d_bad, bad.size(), hipMemcpyDeviceToHost, stream), HEC_ERR_DEVICE);
        HEC_HIP(hipStreamSynchronize(stream), HEC_ERR_DEVICE);

        // ---- phase 2, batched over every stripe with a failed survivor.  A
        // round re-plans each such stripe on the host (drop what failed, take
        // the first k available shards), verifies every newly used cell of
        // every stripe with at most one checksum launch per shard index (a
        // stripe-list launch), and reads the flags back once.  At most m
        // rounds; then one mixed-pattern decode rebuilds every missing or
        // failed data cell of those stripes with its final plan.
        std::vector<uint32_t> F;  // stripes still being repaired
        for (size_t s = 0; s < stripes; s++) {
            bool any = false;
            for (size_t r = 0; r < k; r++) any |= bad[s * n + surv[r]] != 0;
            if (any) F.push_back(uint32_t(s));
        }
        if (F.empty()) return HEC_OK;
        // phase 2 uses the coder's shared device scratch (verify_ws): one
        // verifier at a time, and the stream drained before the lock is
        // released on every path (error returns included), so no queued
        // launch of ours still reads the scratch when another thread grows it
        std::lock_guard<std::mutex> vlk(c->verify_mu);
        struct DrainOnExit {
            hipStream_t s;
            ~DrainOnExit() {
                (void)hipStreamSynchronize(s);
                (void)hipGetLastError();
            }
        } drain_on_exit{stream};
        int status = HEC_OK;
        std::vector<uint8_t> ok(F.size() * n, 0);  // cell verified good
        for (size_t f = 0; f < F.size(); f++)
            for (size_t r = 0; r < k; r++) ok[f * n + surv[r]] = bad[F[f] * n + surv[r]] == 0;
        std::vector<uint8_t> active(F.size(), 1);
        const size_t nck = (cell_len + bytes_per_checksum - 1) / bytes_per_checksum;
        (void)nck;
        for (size_t round = 0; round <= c->m + 1; round++) {
            std::vector<std::vector<uint32_t>> lists(n);
            size_t todo_cells = 0;
            for (size_t f = 0; f < F.size(); f++) {
                if (!active[f]) continue;
                const uint8_t* row = &bad[F[f] * n];
                size_t picked = 0;
                for (size_t i = 0; i < n && picked < k; i++) {
                    if (!present[i] || row[i]) continue;
                    picked++;
                    if (!ok[f * n + i]) {
                        lists[i].push_back(F[f]);
                        todo_cells++;
                    }
                }
                if (picked < k) {  // fewer than k cells left that can verify
                    active[f] = 0;
                    status = HEC_ERR_NOT_ENOUGH_SHARDS;
                }
            }
            if (todo_cells == 0) break;
            // one upload of every list, one launch per shard index, one read-back
            std::vector<uint32_t> flat;
            std::vector<size_t> off(n, 0);
            for (size_t i = 0; i < n; i++) {
                off[i] = flat.size();
                flat.insert(flat.end(), lists[i].begin(), lists[i].end());
            }
            const size_t need = flat.size() * sizeof(uint32_t);
            if (c->verify_ws_bytes < need) {
                // stream-ordered: growing the scratch costs no device-wide sync
                if (c->verify_ws) (void)hipFreeAsync(c->verify_ws, stream);
                c->verify_ws = nullptr;
                c->verify_ws_bytes = 0;
                const size_t want = std::max(need, size_t(64) << 10);
                HEC_HIP(hipMallocAsync(reinterpret_cast<void**>(&c->verify_ws), want, stream), HEC_ERR_NO_MEMORY);
                c->verify_ws_bytes = want;
            }
            const uint32_t* d_lists = reinterpret_cast<const uint32_t*>(c->verify_ws);
            HEC_HIP(hipMemcpyAsync(c->verify_ws, flat.data(), need, hipMemcpyHostToDevice, stream), HEC_ERR_DEVICE);
            for (size_t i = 0; i < n; i++) {
                if (lists[i].empty()) continue;
                const uint8_t* tb[1] = {d_shards[i]};
                const size_t ts[1] = {shard_strides[i]};
                const uint8_t tid[1] = {uint8_t(i)};
                const int rc = checksum_launch(c, kind, tb, ts, tid, 1, n, cell_len, lists[i].size(), bytes_per_checksum,
                                               nullptr, d_sums, d_bad, stream, d_lists + off[i]);
                if (rc != HEC_OK) return rc;
            }
            HEC_HIP(hipMemcpyAsync(bad.data(), d_bad, bad.size(), hipMemcpyDeviceToHost, stream), HEC_ERR_DEVICE);
            HEC_HIP(hipStreamSynchronize(stream), HEC_ERR_DEVICE);  // also keeps `flat` alive through the upload
            for (size_t i = 0; i < n; i++)
                for (uint32_t s : lists[i]) {
                    const size_t f = size_t(std::lower_bound(F.begin(), F.end(), s) - F.begin());
                    ok[f * n + i] = bad[size_t(s) * n + i] == 0;
                }
        }
        // rebuild: final presence mask per repaired stripe, every other stripe
        // a no-op (nothing missing), one mixed-pattern decode launch
        const uint64_t all = n >= 64 ? ~uint64_t(0) : ((uint64_t(1) << n) - 1);
        std::vector<uint64_t> masks(stripes, all);
        bool any_rebuild = false;
        for (size_t f = 0; f < F.size(); f++) {
            if (!active[f]) continue;
            uint64_t mask = 0;
            for (size_t i = 0; i < n; i++)
                if (present[i] && !bad[size_t(F[f]) * n + i]) mask |= uint64_t(1) << i;
            masks[F[f]] = mask;
            any_rebuild = true;
        }
        if (any_rebuild) {
            const size_t ws_need = mixed_workspace(k, c->m, stripes);
            if (c->verify_ws_bytes < ws_need) {
                if (c->verify_ws) (void)hipFreeAsync(c->verify_ws, stream);
                c->verify_ws = nullptr;
                c->verify_ws_bytes = 0;
                HEC_HIP(hipMallocAsync(reinterpret_cast<void**>(&c->verify_ws), ws_need, stream), HEC_ERR_NO_MEMORY);
                c->verify_ws_bytes = ws_need;
            }
            // storage for shard indices no plan reads (absent for the whole batch)
            const uint8_t* shards_all[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
            for (size_t i = 0; i < n; i++) shards_all[i] = d_shards[i] ? d_shards[i] : d_out[0];
            const int rc = mixed_decode_impl(c, shards_all, shard_strides, d_out, out_strides, masks.data(), cell_len,
                                             stripes, c->verify_ws, c->verify_ws_bytes, hip_stream);
            if (rc != HEC_OK) return rc;
        }
        HEC_HIP(hipStreamSynchronize(stream), HEC_ERR_DEVICE);
        return status;
    });
}

// ---- multi-GPU coder group -----------------------------------

}  // extern "C"

struct hec_group {
    std::vector<hec_coder_t*> coders;  // one per slot
};

namespace {

void group_range(size_t total, size_t n, size_t i, size_t* first, size_t* count) {
    const size_t base = total / n, extra = total % n;  // hdfs_native_ec.dist.shard_range
    *first = i * base + std::min(i, extra);
    *count = base + (i < extra ? 1 : 0);
}

// Runs body(slot) for every slot, slots 1.. on their own threads and slot 0 on
// the caller's; returns the lowest failing slot's status and copies its
// hec_last_error() text into the caller's thread.
template <class F>
int group_run(hec_group* g, F&& body) {
    const size_t n = g->coders.size();
    std::vector<int> rc(n, HEC_OK);
    std::vector<std::string> err(n);
    auto run = [&](size_t i) {
        rc[i] = body(i);
        if (rc[i] != HEC_OK) err[i] = g_last_error;
    };
    // Slots whose thread cannot be started run inline after slot 0; every
    // started thread is joined before returning (a joinable std::thread that
    // is destroyed would terminate the process across the ABI).
    std::vector<std::thread> th;
    std::vector<size_t> inline_slots;
    th.reserve(n);
    for (size_t i = 1; i < n; i++) {
        try {
            th.emplace_back(run, i);
        } catch (...) {
            inline_slots.push_back(i);
        }
    }
    run(0);
    for (size_t i : inline_slots) run(i);
    for (auto& t : th) t.join();
    for (size_t i = 0; i < n; i++)
        if (rc[i] != HEC_OK) {
            std::snprintf(g_last_error, sizeof(g_last_error), "group slot %zu: %s", i, err[i].c_str());
            return rc[i];
        }
    return HEC_OK;
}

}  // namespace

extern "C" {

int hec_group_create(const char* codec, size_t data_units, size_t parity_units, const int* devices,
                     size_t n_devices, hec_group_t** out) {
    if (!out) return HEC_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || n_devices == 0 || n_devices > 64) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        auto* g = new hec_group();
        for (size_t i = 0; i < n_devices; i++) {
            hec_coder_t* c = nullptr;
            const int rc = hec_coder_create_codec(codec, data_units, parity_units, devices[i], &c);
            if (rc != HEC_OK) {
                hec_group_destroy(g);
                return rc;
            }
            g->coders.push_back(c);
        }
        *out = g;
        return HEC_OK;
    });
}

void hec_group_destroy(hec_group_t* g) {
    if (!g) return;
    for (auto* c : g->coders) hec_coder_destroy(c);
    delete g;
}

size_t hec_group_size(const hec_group_t* g) { return g ? g->coders.size() : 0; }

hec_coder_t* hec_group_coder(hec_group_t* g, size_t slot) {
    return (g && slot < g->coders.size()) ? g->coders[slot] : nullptr;
}

int hec_group_range(const hec_group_t* g, size_t total, size_t slot, size_t* first, size_t* count) {
    if (!g || !first || !count || slot >= g->coders.size()) return HEC_ERR_INVALID_ARG;
    group_range(total, g->coders.size(), slot, first, count);
    return HEC_OK;
}

int hec_group_encode_host_batch(hec_group_t* g, const uint8_t* h_data, uint8_t* h_parity, size_t cell_len,
                                size_t stripes, size_t chunk_stripes) {
    if (!g || !h_data || !h_parity || cell_len == 0 || chunk_stripes == 0) return HEC_ERR_INVALID_ARG;
    if (stripes == 0) return HEC_OK;
    return guarded([&] {
        return group_run(g, [&](size_t i) {
            hec_coder_t* c = g->coders[i];
            size_t first, count;
            group_range(stripes, g->coders.size(), i, &first, &count);
            if (count == 0) return int(HEC_OK);
            return hec_encode_host_batch(c, h_data + first * c->k * cell_len, h_parity + first * c->m * cell_len,
                                         cell_len, count, chunk_stripes);
        });
    });
}

int hec_group_decode_host_batch(hec_group_t* g, const uint8_t* const* h_vertical, size_t cell_len, size_t rows,
                                uint8_t* h_file, size_t chunk_rows) {
    if (!g || !h_vertical || !h_file || cell_len == 0 || chunk_rows == 0) return HEC_ERR_INVALID_ARG;
    if (rows == 0) return HEC_OK;
    return guarded([&] {
        return group_run(g, [&](size_t i) {
            hec_coder_t* c = g->coders[i];
            size_t first, count;
            group_range(rows, g->coders.size(), i, &first, &count);
            if (count == 0) return int(HEC_OK);
            const uint8_t* vert[HEC_MAX_DATA_UNITS + HEC_MAX_PARITY_UNITS];
            for (size_t s = 0; s < c->k + c->m; s++)
                vert[s] = h_vertical[s] ? h_vertical[s] + first * cell_len : nullptr;
            return hec_decode_host_batch(c, vert, cell_len, count, h_file + first * c->k * cell_len, chunk_rows);
        });
    });
}

}  // extern "C"

// Device-resident batches over the group: every slot's launch is enqueued
// from the calling thread (an enqueue is microseconds and asynchronous, so
// the GPUs run concurrently without host threads); every slot is tried, the
// lowest failing slot's status is returned.
namespace {
template <class F>
int group_enqueue(hec_group_t* g, F&& body) {
    int first_rc = HEC_OK;
    size_t first_slot = 0;
    std::string first_err;
    for (size_t i = 0; i < g->coders.size(); i++) {
        const int rc = body(i);
        if (rc != HEC_OK && first_rc == HEC_OK) {
            first_rc = rc;
            first_slot = i;
            first_err = g_last_error;
        }
    }
    if (first_rc != HEC_OK)
        std::snprintf(g_last_error, sizeof(g_last_error), "group slot %zu: %s", first_slot, first_err.c_str());
    return first_rc;
}
}  // namespace

extern "C" {

int hec_group_encode_device(hec_group_t* g, const uint8_t* const* d_data, const size_t* data_strides,
                            uint8_t* const* d_parity, const size_t* parity_strides, size_t cell_len,
                            const size_t* stripes, void* const* hip_streams) {
    if (!g || !d_data || !data_strides || !d_parity || !parity_strides || !stripes || cell_len == 0)
        return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        return group_enqueue(g, [&](size_t i) {
            hec_coder_t* c = g->coders[i];
            if (stripes[i] == 0) return int(HEC_OK);
            return hec_encode_device(c, d_data + i * c->k, data_strides + i * c->k, d_parity + i * c->m,
                                     parity_strides + i * c->m, cell_len, stripes[i],
                                     hip_streams ? hip_streams[i] : nullptr);
        });
    });
}

int hec_group_decode_device(hec_group_t* g, const uint8_t* const* d_shards, const size_t* shard_strides,
                            uint8_t* const* d_out, const size_t* out_strides, size_t cell_len,
                            const size_t* stripes, void* const* hip_streams) {
    if (!g || !d_shards || !shard_strides || !d_out || !out_strides || !stripes || cell_len == 0)
        return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        return group_enqueue(g, [&](size_t i) {
            hec_coder_t* c = g->coders[i];
            if (stripes[i] == 0) return int(HEC_OK);
            const size_t n = c->k + c->m;
            return hec_decode_device(c, d_shards + i * n, shard_strides + i * n, d_out + i * c->k,
                                     out_strides + i * c->k, cell_len, stripes[i],
                                     hip_streams ? hip_streams[i] : nullptr);
        });
    });
}

int hec_device_alloc(int device, size_t bytes, unsigned flags, void** out) {
    if (!out || bytes == 0 || (flags & ~unsigned(HEC_ALLOC_CONTIGUOUS))) return HEC_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded([&] {
        DeviceGuard g(device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        const unsigned hf = (flags & HEC_ALLOC_CONTIGUOUS) ? hipDeviceMallocContiguous : hipDeviceMallocDefault;
        HEC_HIP(hipExtMallocWithFlags(out, bytes, hf), HEC_ERR_NO_MEMORY);
        return HEC_OK;
    });
}

int hec_device_free(int device, void* ptr) {
    if (!ptr) return HEC_OK;
    return guarded([&] {
        DeviceGuard g(device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        HEC_HIP(hipFree(ptr), HEC_ERR_DEVICE);
        return HEC_OK;
    });
}

int hec_device_copy(int device, void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return HEC_OK;
    if (!dst || !src) return HEC_ERR_INVALID_ARG;
    return guarded([&] {
        DeviceGuard g(device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        HEC_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault), HEC_ERR_DEVICE);
        return HEC_OK;
    });
}

int hec_device_synchronize(int device, void* hip_stream) {
    return guarded([&] {
        DeviceGuard g(device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        HEC_HIP(hipStreamSynchronize(static_cast<hipStream_t>(hip_stream)), HEC_ERR_DEVICE);
        return HEC_OK;
    });
}

// ---- NUMA-placed pinned host buffers -------------------------------------

namespace {

std::mutex g_host_mu;
std::unordered_map<void*, size_t> g_host_allocs;  // ptr -> mapped bytes

int numa_node_of(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
    std::string id(bus);
    for (auto& ch : id) ch = char(std::tolower(static_cast<unsigned char>(ch)));
    std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
    int node = -1;
    if (!(f >> node)) return -1;
    return node;
}

}  // namespace

void hec_queue_stats(int device, uint64_t* streams, uint64_t* graph_sets, int* keyed_by_id) {
    if (streams) *streams = 0;
    if (graph_sets) *graph_sets = 0;
    if (keyed_by_id) *keyed_by_id = 0;
    try {
        int n = 0;
        if (device < 0 || hipGetDeviceCount(&n) != hipSuccess || device >= n) {
            (void)hipGetLastError();
            return;  // no such device: zeros, and no per-device state created
        }
        hec::queue_stats(device, streams, graph_sets);
        if (keyed_by_id) *keyed_by_id = hec::queue_keyed_by_id();
    } catch (...) {
        if (streams) *streams = 0;
        if (graph_sets) *graph_sets = 0;
    }
}

int hec_device_numa_node(int device) {
    try {
        return numa_node_of(device);
    } catch (...) {
        return -1;
    }
}

int hec_host_alloc(int device, size_t bytes, int numa_node, void** out) {
    if (!out || bytes == 0 || numa_node < -1 || numa_node >= 1024) return HEC_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded([&] {
        DeviceGuard g(device);
        if (!g.ok) return fail(HEC_ERR_DEVICE, "hipSetDevice", hipErrorInvalidDevice);
        const int node = numa_node >= 0 ? numa_node : numa_node_of(device);
        const size_t page = size_t(sysconf(_SC_PAGESIZE));
        const size_t len = (bytes + page - 1) / page * page;
        void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return int(HEC_ERR_NO_MEMORY);
        if (node >= 0) {
            // MPOL_BIND to the node before the pages exist: every page is
            // faulted in there by the touch below
            unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
            mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
            const long MPOL_BIND_ = 2;
            if (syscall(SYS_mbind, p, len, MPOL_BIND_, mask, 1024ul, 0ul) != 0) {
                munmap(p, len);
                std::snprintf(g_last_error, sizeof(g_last_error), "mbind to NUMA node %d failed", node);
                return int(HEC_ERR_INVALID_ARG);
            }
        }
        std::memset(p, 0, len);
        const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
        if (e != hipSuccess) {
            munmap(p, len);
            (void)hipGetLastError();
            return fail(HEC_ERR_NO_MEMORY, "hipHostRegister", e);
        }
        std::lock_guard<std::mutex> lk(g_host_mu);
        g_host_allocs[p] = len;
        *out = p;
        return int(HEC_OK);
    });
}

int hec_host_free(void* ptr) {
    if (!ptr) return HEC_OK;
    return guarded([&] {
        size_t len = 0;
        {
            std::lock_guard<std::mutex> lk(g_host_mu);
            auto it = g_host_allocs.find(ptr);
            if (it == g_host_allocs.end()) return int(HEC_ERR_INVALID_ARG);
            len = it->second;
            g_host_allocs.erase(it);
        }
        (void)hipHostUnregister(ptr);
        (void)hipGetLastError();
        munmap(ptr, len);
        return int(HEC_OK);
    });
}

#ifdef HEC_EXPERIMENTAL
// Measurement knobs (include/hdfs_ec_amd_exp.h): the HEC_EXPERIMENTAL build
// only.  The product library has no knobs and does not export this symbol.
int hec_tune_set(int key, int value) {
    const int rc = hec::tune_store(key, value);
    if (rc != HEC_OK)
        std::snprintf(g_last_error, sizeof(g_last_error), "hec_tune_set: key %d value %d unknown or out of range", key,
                      value);
    return rc;
}
#endif

}  // extern "C"
