// jit.hpp -- plan-time specialisation of the fused decode + verify kernel.
//
// The decode + verify kernel (ec_fused_kernel.hpp, VERIFY = true) rebuilds the
// missing data rows from the k survivors while it checksums them.  Its matrix
// is the decode plan's, known only at run time, so the ahead-of-time build
// runs it through the v_perm product tables (PermNet): 5 selector ops per
// input dword + 3 v_perm + 2 XOR per (dword, row), 960 VALU per 8 dwords of
// every survivor for RS(6,3) with 3 rows lost.  For a plan the engine meets
// it generates that matrix's bit-sliced XOR network (xor_net.hpp: 231 XOR-type
// ops per 8-dword group for the same plan, + 48-op transposes per cell) and
// compiles the same kernel template with it through hiprtc: the kernel
// becomes as cheap in VALU as the bit-sliced encode + CRC.
//
// The compile takes seconds, so by default it runs on a background thread the
// first time a plan is seen; launches use the ahead-of-time kernel until the
// specialised one is ready (the results are identical either way: both are
// checked against the oracle).  hec_coder_prepare_decode compiles
// synchronously.  Code objects are cached per process and on disk.
//   HEC_JIT=0      never specialise (ahead-of-time kernels only)
//   HEC_JIT=sync   compile on first use, synchronously
//   HEC_JIT_CACHE  code-object cache directory ("" = none; default
//                  $XDG_CACHE_HOME or ~/.cache, /hdfs_ec_amd/jit)
// hiprtc is loaded with dlopen: without it the engine runs the ahead-of-time
// kernels only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace hec {
namespace jit {

struct VerifyKernel {
    hipFunction_t fn = nullptr;
};

// The specialised decode + verify kernel of the fused launch shape for (k,
// e rows, checksum kind, matrix = e x k row-major) on `device` (the current
// device), or false: JIT off or unavailable, shape not covered, compile
// queued / running / failed.  wait = compile now (synchronously) if needed.
// slabs = the launch shape (KiB of every cell per wave: 8, or 4 with the
// inputs two at a time); default_slabs(k, e) is the specialised kernel's
// default (4: measured faster than 8 for every plan tried), which may differ
// from the ahead-of-time kernel's (8 at k <= 6, e <= 3).
// wpe = waves per SIMD (2, or 3 at 4 slabs: one 768-thread block per CU);
// pfd = load schedule (1 default; measurement shapes: pick_pfd).
// scheme = the CRC lookup scheme (12 default; 15 = slicing-by-32 tail,
// CRC32C only, measurement build)
// wq = tiles from the work queue of wave-tiles (work_queue.hpp): the
// launch then needs a.queue and the per-wave tile geometry (ec_fused.hip)
bool verify_kernel(int device, int k, int e, int kind, int slabs, int wpe, int pfd, const uint8_t* matrix, bool wait,
                   VerifyKernel* out, int scheme = 12, bool wq = false);
// whether the specialised decode + verify of (k, e) takes the work queue
// (launch and prepare must agree: ec_fused.hip, hec_coder_prepare_decode)
bool default_wq(int k, int e);
int default_slabs(int k, int e);
int default_pfd(int k, int e);
// the pfd a measurement-build tune key 24 value asks for at this slab count
// (2 at 4 slabs, 3 at 8, 4 and 5 at either; anything else: default_pfd)
int pick_pfd(int key, int slabs, int k, int e);

// Compiles (or loads from the disk cache) the specialised kernel's code
// object without a device: warms the caches ahead of use.  False when the
// shape is not covered or the compile failed.
bool warm(int k, int e, int kind, int slabs, int wpe, int pfd, const uint8_t* matrix, int scheme = 12, bool wq = false);

// Counters for tests and the bench line: kernels compiled (or loaded from
// the disk cache), compiles failed, launches that used a specialised kernel.
struct Stats {
    uint64_t compiled, from_disk, failed, launches;
    double compile_seconds;  // total wall time in hiprtc
};
Stats stats();
void count_launch();

// Generated source of the specialised kernel (tests / inspection).
size_t verify_source(int k, int e, int kind, const uint8_t* matrix, char* buf, size_t len);

}  // namespace jit
}  // namespace hec
