// jit.cpp -- plan-time specialisation of the fused decode + verify kernel
// (see jit.hpp): network generation (xor_net.hpp), hiprtc compile of
// ec_fused_kernel.hpp with it, code-object caches, module load per device.
#include "jit.hpp"

#ifndef _GNU_SOURCE
#define _GNU_SOURCE  // dlmopen
#endif
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "xor_net.hpp"

namespace hec {
namespace jit {

namespace {

// The kernel headers, embedded at build time (Makefile: build/jit_headers.inc)
// so that the library compiles its kernels without its source tree.
#include "jit_headers.inc"

// ---- hiprtc, loaded on first use -----------------------------------------
// (the subset of hip/hiprtc.h the JIT calls; hiprtcResult 0 = success)
typedef struct ihiprtcProgram* hiprtcProgram;
struct Rtc {
    bool ok = false;
    int (*create)(hiprtcProgram*, const char*, const char*, int, const char* const*, const char* const*);
    int (*compile)(hiprtcProgram, int, const char* const*);
    int (*log_size)(hiprtcProgram, size_t*);
    int (*log)(hiprtcProgram, char*);
    int (*code_size)(hiprtcProgram, size_t*);
    int (*code)(hiprtcProgram, char*);
    int (*destroy)(hiprtcProgram*);
    int (*add_name)(hiprtcProgram, const char*);
    int (*lowered)(hiprtcProgram, const char*, const char**);
    int (*version)(int*, int*);
};

const Rtc& rtc() {
    static Rtc r = [] {
        Rtc t;
        // The ROCm install's hiprtc, in a link-map namespace of its own: a
        // process that already holds another HIP stack (PyTorch wheels bundle
        // their own libhiprtc / libamd_comgr) would otherwise resolve both to
        // the bundled copies -- an older compiler than the one that built
        // this library, which spills more registers in this kernel.
        const char* root = std::getenv("ROCM_PATH");
        const std::string lib = std::string(root && *root ? root : "/opt/rocm") + "/lib/libhiprtc.so.7";
        void* h = dlmopen(LM_ID_NEWLM, lib.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_LOCAL);
        if (!h) return t;
        auto sym = [&](const char* n) { return dlsym(h, n); };
        t.create = reinterpret_cast<decltype(t.create)>(sym("hiprtcCreateProgram"));
        t.compile = reinterpret_cast<decltype(t.compile)>(sym("hiprtcCompileProgram"));
        t.log_size = reinterpret_cast<decltype(t.log_size)>(sym("hiprtcGetProgramLogSize"));
        t.log = reinterpret_cast<decltype(t.log)>(sym("hiprtcGetProgramLog"));
        t.code_size = reinterpret_cast<decltype(t.code_size)>(sym("hiprtcGetCodeSize"));
        t.code = reinterpret_cast<decltype(t.code)>(sym("hiprtcGetCode"));
        t.destroy = reinterpret_cast<decltype(t.destroy)>(sym("hiprtcDestroyProgram"));
        t.add_name = reinterpret_cast<decltype(t.add_name)>(sym("hiprtcAddNameExpression"));
        t.lowered = reinterpret_cast<decltype(t.lowered)>(sym("hiprtcGetLoweredName"));
        t.version = reinterpret_cast<decltype(t.version)>(sym("hiprtcVersion"));
        t.ok = t.create && t.compile && t.log_size && t.log && t.code_size && t.code && t.destroy && t.add_name &&
               t.lowered && t.version;
        return t;
    }();
    return r;
}

enum class Mode { kOff, kAsync, kSync };

Mode mode() {
    static const Mode m = [] {
        const char* v = std::getenv("HEC_JIT");
        if (v && (std::strcmp(v, "0") == 0 || std::strcmp(v, "off") == 0)) return Mode::kOff;
        if (v && std::strcmp(v, "sync") == 0) return Mode::kSync;
        return Mode::kAsync;
    }();
    return m;
}

// slabs = KiB of every cell per wave (ec_fused.hip): 8, or 4 with the
// inputs taken two at a time
// shape: sl = slabs (8, or 4 with inputs in pairs), wpe = waves per SIMD (2,
// or 3 at 4 slabs: one 768-thread block per CU), pfd = input pairs loaded
// ahead (4 slabs: 1 or 2) or 3 = loads issued before the parity math (8 slabs)
// or 4 = one pair / input ahead with the expected sums prefetched per tile,
// 5 = the rebuilt rows stored and the next tile's first inputs loaded before
// the last CRC round
struct Shape {
    int slabs, wpe, pfd;
    int scheme = 12;  // CRC lookup scheme: 12 (the fold + 11-bit tail), 15 (slicing-by-32 tail; CRC32C)
    bool wq = false;  // tiles from the work queue of wave-tiles (work_queue.hpp)
};

std::string kernel_name(int k, int e, int kind, Shape sh) {
    return "hec::gf_fused_crc<" + std::to_string(k) + ", " + std::to_string(e) + ", " + std::to_string(sh.slabs) +
           ", " + std::to_string(sh.scheme) + ", " + std::to_string(kind) + ", true, " + std::to_string(sh.wpe) + ", " +
           (sh.slabs == 4 ? "true" : "false") + ", hec::jit_plan::Net, " + std::to_string(sh.pfd) +
           (sh.wq ? ", true>" : ">");
}

bool shape_ok(int k, int e, int kind, Shape sh) {
    return (k == 2 || k == 3 || k == 6 || k == 10) && e >= 1 && e <= 4 && (kind == 0 || kind == 1) &&
           (sh.slabs == 4 || sh.slabs == 8) && (sh.wpe == 2 || (sh.wpe == 3 && sh.slabs == 4)) &&
           (sh.pfd == 1 || (sh.pfd == 2 && sh.slabs == 4) || (sh.pfd == 3 && sh.slabs == 8) || sh.pfd == 4 || sh.pfd == 5) &&
           (sh.scheme == 12 || (sh.scheme == 15 && kind == 0));
}

std::string entry_key(const std::string& arch, int k, int e, int kind, Shape sh, const uint8_t* matrix) {
    std::string key = arch + "/" + std::to_string(k) + "/" + std::to_string(e) + "/" + std::to_string(kind) + "/" +
                      std::to_string(sh.slabs) + "/" + std::to_string(sh.wpe) + "/" + std::to_string(sh.pfd) + "/" +
                      std::to_string(sh.scheme) + (sh.wq ? "/q/" : "/");
    key.append(reinterpret_cast<const char*>(matrix), size_t(e) * k);
    return key;
}

std::string make_source(int k, int e, int kind, const uint8_t* matrix) {
    const auto nets = xornet::matrix_network(matrix, e, k);
    std::string s;
    s += "// generated by jit.cpp: decode + verify, k = " + std::to_string(k) + ", rows = " + std::to_string(e) +
         ", checksum kind " + std::to_string(kind) + ", " + std::to_string(xornet::network_ops(nets)) +
         " XOR-type ops per 8-dword group\n// matrix:";
    for (int j = 0; j < e; j++) {
        s += " [";
        for (int i = 0; i < k; i++) s += (i ? "," : "") + std::to_string(matrix[j * k + i]);
        s += "]";
    }
    s += "\n#include \"ec_fused_kernel.hpp\"\n\nnamespace hec {\nnamespace jit_plan {\n\n";
    const std::string acc = "uint32_t (&acc)[" + std::to_string(8 * e) + "]";
    s += "struct Net {\n    static constexpr bool kBsl = true;\n    template <int I>\n"
         "    __device__ static void absorb(const uint32_t (&p)[8], " + acc + ");\n"
         "    __device__ static void absorb_at(int i, const uint32_t (&p)[8], " + acc + ");\n};\n\n";
    for (int i = 0; i < k; i++) s += xornet::emit_input(nets[i], i, e) + "\n";
    s += "__device__ __forceinline__ void Net::absorb_at(int i, const uint32_t (&p)[8], " + acc + ") {\n"
         "    switch (i) {\n";
    for (int i = 0; i < k; i++)
        s += "        case " + std::to_string(i) + ": absorb<" + std::to_string(i) + ">(p, acc); break;\n";
    s += "        default: break;\n    }\n}\n\n}  // namespace jit_plan\n}  // namespace hec\n";
    return s;
}

constexpr uint32_t kCacheMagic = 0x32434548u;  // "HEC2": the checked disk-cache format

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

std::string cache_dir() {
    const char* v = std::getenv("HEC_JIT_CACHE");
    if (v) return v;  // "" = no disk cache
    const char* x = std::getenv("XDG_CACHE_HOME");
    const char* home = std::getenv("HOME");
    std::string base = x && *x ? x : (home && *home ? std::string(home) + "/.cache" : "");
    return base.empty() ? "" : base + "/hdfs_ec_amd/jit";
}

void mkdirs(const std::string& d) {
    for (size_t i = 1; i <= d.size(); i++)
        if (i == d.size() || d[i] == '/') (void)mkdir(d.substr(0, i).c_str(), 0755);
}

// The gfx target a device's code object is compiled for (its gcnArchName up
// to the first ':'), cached per device; without a device (hec_jit_warm on a
// build host) $HEC_JIT_ARCH, else gfx950.  Part of the entry and disk-cache
// keys, so a code object is never loaded on a device of another target.
std::string device_arch(int device) {
    static std::mutex mu;
    static std::map<int, std::string> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(device);
    if (it != cache.end()) return it->second;
    std::string arch;
    hipDeviceProp_t p;
    if (device >= 0 && hipGetDeviceProperties(&p, device) == hipSuccess) {
        arch = p.gcnArchName;
        arch = arch.substr(0, arch.find(':'));
    } else {
        (void)hipGetLastError();
    }
    if (arch.empty()) {
        const char* v = std::getenv("HEC_JIT_ARCH");
        arch = v && *v ? v : "gfx950";
    }
    return cache[device] = arch;
}

// hiprtc options past the arch (part of the disk-cache key)
constexpr const char* kRtcOptions = "-O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None";

enum class State { kQueued, kCompiling, kReady, kFailed };

struct Entry {
    int k = 0, e = 0, kind = 0;
    std::string arch;  // gfx target (device_arch)
    Shape shape{8, 2, 1};
    std::vector<uint8_t> matrix;
    State state = State::kQueued;
    std::vector<char> code;        // code object (once kReady)
    std::string lowered;           // mangled kernel name
    std::map<int, hipFunction_t> fn;  // per device (module loaded once per device)
    std::map<int, hipModule_t> mod;
};

struct Jit {
    std::mutex mu;
    std::condition_variable cv;        // job queue / state changes
    std::map<std::string, std::shared_ptr<Entry>> entries;
    std::deque<std::shared_ptr<Entry>> queue;
    std::thread worker;
    bool stop = false;
    std::atomic<uint64_t> compiled{0}, from_disk{0}, failed{0}, launches{0};
    std::atomic<uint64_t> compile_ns{0};

    ~Jit() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            queue.clear();
        }
        cv.notify_all();
        if (worker.joinable()) worker.join();  // at most the compile in flight
        // modules are not unloaded: the HIP runtime may already be gone at exit
    }

    void start_worker() {  // under mu
        if (worker.joinable()) return;
        worker = std::thread([this] {
            for (;;) {
                std::shared_ptr<Entry> job;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || !queue.empty(); });
                    if (stop) return;
                    job = queue.front();
                    queue.pop_front();
                    job->state = State::kCompiling;
                }
                build(*job);
            }
        });
    }

    // compile (or load from disk) one entry's code object; sets kReady / kFailed
    void build(Entry& en) {
        const std::string src = make_source(en.k, en.e, en.kind, en.matrix.data());
        const std::string name = kernel_name(en.k, en.e, en.kind, en.shape);
        const Rtc& r = rtc();
        int maj = 0, mnr = 0;
        if (r.ok) r.version(&maj, &mnr);
        const std::string dir = cache_dir();
        const uint64_t h = fnv1a(name + "\n" + en.arch + "\n" + std::to_string(maj) + "." + std::to_string(mnr) +
                                 "\n" + kRtcOptions + "\n" + src + kHeaderDigest);
        char hex[17];
        std::snprintf(hex, sizeof hex, "%016llx", static_cast<unsigned long long>(h));
        const std::string path = dir.empty() ? "" : dir + "/dv-" + hex + ".co";
        std::vector<char> code;
        std::string lowered;
        // disk cache: [magic u32][name length u32][lowered name][code size u64]
        // [fnv1a of the code u64][code object]; a file that does not check out
        // (truncated by a full disk, another format) is ignored and rewritten
        if (!path.empty()) {
            if (FILE* f = std::fopen(path.c_str(), "rb")) {
                uint32_t magic = 0, n = 0;
                uint64_t size = 0, sum = 0;
                if (std::fread(&magic, 4, 1, f) == 1 && magic == kCacheMagic && std::fread(&n, 4, 1, f) == 1 &&
                    n < 4096) {
                    lowered.resize(n);
                    if (std::fread(&lowered[0], 1, n, f) == n && std::fread(&size, 8, 1, f) == 1 &&
                        std::fread(&sum, 8, 1, f) == 1 && size >= 64 && size < (uint64_t(1) << 30)) {
                        code.resize(size);
                        if (std::fread(code.data(), 1, size, f) != size || std::fgetc(f) != EOF ||
                            fnv1a(std::string(code.data(), code.size())) != sum)
                            code.clear();
                    }
                }
                std::fclose(f);
            }
        }
        const bool disk = !code.empty();
        if (!disk && r.ok) {
            const auto t0 = std::chrono::steady_clock::now();
            hiprtcProgram prog = nullptr;
            if (r.create(&prog, src.c_str(), "hec_decode_verify_jit.hip", kNumHeaders, kHeaderTexts, kHeaderNames) ==
                0) {
                const std::string expr = "&" + name;
                r.add_name(prog, expr.c_str());
                const std::string arch_opt = "--offload-arch=" + en.arch;
                // the ahead-of-time library's flags (Makefile): the work queue's
                // one-lane fetch must not become a wave-combined atomic waited
                // for at issue
                const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17", "-mllvm",
                                      "-amdgpu-atomic-optimizer-strategy=None"};
                if (r.compile(prog, 5, opts) == 0) {
                    size_t n = 0;
                    const char* low = nullptr;
                    if (r.code_size(prog, &n) == 0 && n > 0 && r.lowered(prog, expr.c_str(), &low) == 0 && low) {
                        code.resize(n);
                        lowered = low;
                        if (r.code(prog, code.data()) != 0) code.clear();
                    }
                } else if (std::getenv("HEC_JIT_LOG")) {
                    size_t n = 0;
                    r.log_size(prog, &n);
                    std::string log(n, '\0');
                    if (n) r.log(prog, &log[0]);
                    std::fprintf(stderr, "hec jit: compile failed for %s:\n%s\n", name.c_str(), log.c_str());
                }
                r.destroy(&prog);
            }
            compile_ns += uint64_t(
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
            if (!code.empty() && !path.empty()) {  // write-then-rename: readers never see a partial file
                mkdirs(dir);
                const std::string tmp = path + ".tmp" + std::to_string(getpid());
                if (FILE* f = std::fopen(tmp.c_str(), "wb")) {
                    const uint32_t magic = kCacheMagic, n = uint32_t(lowered.size());
                    const uint64_t size = code.size(), sum = fnv1a(std::string(code.data(), code.size()));
                    bool ok = std::fwrite(&magic, 4, 1, f) == 1 && std::fwrite(&n, 4, 1, f) == 1 &&
                              std::fwrite(lowered.data(), 1, n, f) == n && std::fwrite(&size, 8, 1, f) == 1 &&
                              std::fwrite(&sum, 8, 1, f) == 1 && std::fwrite(code.data(), 1, size, f) == size;
                    ok = std::fclose(f) == 0 && ok;  // a short write surfaces at fclose (full disk)
                    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
                }
            }
        }
        std::lock_guard<std::mutex> lk(mu);
        if (!code.empty()) {
            en.code = std::move(code);
            en.lowered = std::move(lowered);
            en.state = State::kReady;
            (disk ? from_disk : compiled)++;
        } else {
            en.state = State::kFailed;
            failed++;
        }
        cv.notify_all();
    }
};

Jit& jit() {
    static Jit j;
    return j;
}

}  // namespace

bool verify_kernel(int device, int k, int e, int kind, int slabs, int wpe, int pfd, const uint8_t* matrix, bool wait,
                   VerifyKernel* out, int scheme, bool wq) {
    const Shape sh{slabs, wpe, pfd, scheme, wq};
    if (mode() == Mode::kOff || !shape_ok(k, e, kind, sh)) return false;
    if (!rtc().ok && cache_dir().empty()) return false;
    wait = wait || mode() == Mode::kSync;
    const std::string arch = device_arch(device);
    const std::string key = entry_key(arch, k, e, kind, sh, matrix);
    Jit& J = jit();
    std::shared_ptr<Entry> en;
    {
        std::unique_lock<std::mutex> lk(J.mu);
        auto it = J.entries.find(key);
        if (it == J.entries.end()) {
            en = std::make_shared<Entry>();
            en->k = k;
            en->e = e;
            en->kind = kind;
            en->arch = arch;
            en->shape = sh;
            en->matrix.assign(matrix, matrix + size_t(e) * k);
            J.entries.emplace(key, en);
            if (!wait) {
                J.queue.push_back(en);
                J.start_worker();
                J.cv.notify_all();
                return false;
            }
            en->state = State::kCompiling;
        } else {
            en = it->second;
            if (en->state == State::kQueued && wait) {  // take it off the queue, compile here
                for (auto q = J.queue.begin(); q != J.queue.end(); ++q)
                    if (*q == en) {
                        J.queue.erase(q);
                        break;
                    }
                en->state = State::kCompiling;
                lk.unlock();
                J.build(*en);
                lk.lock();
            } else if (en->state == State::kCompiling && wait) {
                J.cv.wait(lk, [&] { return en->state == State::kReady || en->state == State::kFailed; });
            }
            if (en->state != State::kReady) return false;
            auto f = en->fn.find(device);
            if (f != en->fn.end()) {
                out->fn = f->second;
                return true;
            }
        }
    }
    if (en->state == State::kCompiling) J.build(*en);  // a new entry compiled synchronously
    std::lock_guard<std::mutex> lk(J.mu);
    if (en->state != State::kReady) return false;
    auto f = en->fn.find(device);
    if (f == en->fn.end()) {  // first use on this device: load the code object
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr;
        if (hipModuleLoadData(&mod, en->code.data()) != hipSuccess ||
            hipModuleGetFunction(&fn, mod, en->lowered.c_str()) != hipSuccess) {
            (void)hipGetLastError();
            if (mod) (void)hipModuleUnload(mod);
            en->state = State::kFailed;
            J.failed++;
            return false;
        }
        en->mod[device] = mod;
        f = en->fn.emplace(device, fn).first;
    }
    out->fn = f->second;
    return true;
}

bool warm(int k, int e, int kind, int slabs, int wpe, int pfd, const uint8_t* matrix, int scheme, bool wq) {
    const Shape sh{slabs, wpe, pfd, scheme, wq};
    if (!shape_ok(k, e, kind, sh)) return false;
    const std::string arch = device_arch(-1);  // no device: $HEC_JIT_ARCH or gfx950
    const std::string key = entry_key(arch, k, e, kind, sh, matrix);
    Jit& J = jit();
    std::shared_ptr<Entry> en;
    {
        std::unique_lock<std::mutex> lk(J.mu);
        auto it = J.entries.find(key);
        if (it != J.entries.end()) {
            en = it->second;
            if (en->state == State::kQueued) {
                for (auto q = J.queue.begin(); q != J.queue.end(); ++q)
                    if (*q == en) {
                        J.queue.erase(q);
                        break;
                    }
            } else {
                J.cv.wait(lk, [&] { return en->state == State::kReady || en->state == State::kFailed; });
                return en->state == State::kReady;
            }
        } else {
            en = std::make_shared<Entry>();
            en->k = k;
            en->e = e;
            en->kind = kind;
            en->arch = arch;
            en->shape = sh;
            en->matrix.assign(matrix, matrix + size_t(e) * k);
            J.entries.emplace(key, en);
        }
        en->state = State::kCompiling;
    }
    J.build(*en);
    std::lock_guard<std::mutex> lk(J.mu);
    return en->state == State::kReady;
}

Stats stats() {
    Jit& J = jit();
    return Stats{J.compiled.load(), J.from_disk.load(), J.failed.load(), J.launches.load(), J.compile_ns.load() * 1e-9};
}

void count_launch() { jit().launches++; }

// 4 slabs with the inputs in pairs: RS(6,3) {0,1,2} 1.747-1.774 ms against
// 1.804-1.809 at 8 slabs, same box, 3 alternations (profiles/r04h/)
int default_slabs(int, int) { return 4; }
// The specialised decode + verify takes the work queue of wave-tiles (round
// 5).  Same process and buffers, decode of data 0..m-1 + verify of the k
// survivors, 2 sets x 5 alternated rounds (scripts/probe_fused_wq.py,
// profiles/r05af): RS(6,3) x 1024 0.728-0.740 of HBM peak vs 0.685-0.725 in
// block tiles, RS(10,4) x 256 0.667-0.669 vs 0.619-0.620, RS(3,2) x 1024
// 0.691-0.701 vs 0.648-0.674.
bool default_wq(int, int) { return true; }
int default_pfd(int, int) { return 1; }

int pick_pfd(int key, int slabs, int k, int e) {
    if (key == 2 && slabs == 4) return 2;
    if (key == 3 && slabs == 8) return 3;
    if (key == 4 || key == 5) return key;
    return default_pfd(k, e);
}

size_t verify_source(int k, int e, int kind, const uint8_t* matrix, char* buf, size_t len) {
    const std::string s = make_source(k, e, kind, matrix);
    if (buf && len) {
        const size_t n = std::min(len - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = '\0';
    }
    return s.size() + 1;
}

}  // namespace jit
}  // namespace hec
