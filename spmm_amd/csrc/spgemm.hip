// spgemm.hip -- libmi355_spgemm.so: the C ABI declared in include/spgemm.h.
//
// Host side of the engine: argument checking, workspace carving, algorithm sequencing
// (ALG1 single pass, ALG2 two phase, ALG3 chunked two phase) and type dispatch to the
// kernels in spgemm_kernels.hpp.  No HIP or C++ type crosses the ABI.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "spgemm.h"
#include "spgemm_kernels.hpp"
#include "spgemm_tile.hpp"
#include "spgemm_tile_dn.hpp"
#include "spgemm_spmv.hpp"
#include "spgemm_row.hpp"

using namespace spg;

constexpr int PINNED_WORDS = MIRROR_GEN_WORD + 1;   // host-pinned: 16 scalars, per-chunk spill counts, generation

struct spg_handle_s {
    int device = 0;
    int cus = 256;                  // compute units (persistent grids)
    hipStream_t stream = nullptr;
    int last_hip = 0;
    int64_t* pinned = nullptr;      // PINNED_WORDS host-pinned int64 for device->host scalars
    int64_t mirror_gen = 0;         // generation of the last scan that mirrors into `pinned`
    int32_t* spill_ctr = nullptr;   // ALG1 on k_row: spill counter, re-armed by the scan kernel
    bool spill_ctr_dirty = false;   // a count pass ran without its scan (re-zero first)
    // bound of the ALG1 numeric launch's waits (scan look-back, 64-row group words), wall-clock
    // ticks; a wait past it computes the prefix directly (same result).  SPG_LB_SPIN_TICKS
    // (read once per handle) lowers it -- 0 sends every wait to that path, which the GPU
    // tests use to check it bit for bit; it cannot change any result.
    uint64_t lb_spin = SCAN_SPIN;
    // the ordered-LDS property k_tile_dn / k_tile_sp rely on (same-address lanes of one
    // ds_add_f64 apply in ascending lane order, DS ops in issue order), checked on the device
    // at spg_create (lds_order_check); false sends fp64 tiles to k_tile's owner rounds, which
    // need neither.  SPG_LDS_ORDERED=0 forces false (a schedule-only switch, for the tests).
    bool lds_ordered = true;
    bool lds_ordered32 = true;      // the same for ds_add_f32 (the fp32 entry runs' third-and-later runs)
    void* scratch = nullptr;        // internal device scratch (plan-time analysis)
    size_t scratch_bytes = 0;
    // per-phase timing (spg_set_timing / spg_get_timing)
    bool timing = false;
    struct Pending { int phase; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    double ms[SPG_NUM_PHASES] = {};
    int64_t launches[SPG_NUM_PHASES] = {};
    // what the last size query measured (see spg_plan)
    bool q_valid = false;
    spg_csr_t q_A{}, q_B{};
    spg_alg_t q_alg = SPG_ALG2;
    float q_cf = 0.f;
    int64_t q_P = -1, q_seg_len = 0;
    std::vector<int64_t> q_chunk_rows, q_chunk_nz;
};

struct spg_plan_s {
    spg_csr_t A{}, B{};
    spg_alg_t alg = SPG_ALG2;
    float cf = 0.2f;
    char* ws = nullptr;
    size_t ws_bytes = 0;
    // workspace carve
    int64_t* scalars = nullptr;     // [0] total, [1] overflow, [2..] flags
    int64_t* row_cnt = nullptr;     // rows
    uint32_t* seg = nullptr;        // 2 * seg_len
    int64_t seg_len = 0;
    int64_t* ub = nullptr;          // ALG1: product prefix, rows + 1
    int32_t* tj = nullptr;          // ALG1: upper-bound column buffer (P entries)
    void* tx = nullptr;             // ALG1: upper-bound value buffer (P entries)
    int64_t P = -1;                 // number of products, -1 until known
    int64_t nnzC = -1;
    void* c_indptr = nullptr;
    spg_index_t c_indptr_type = SPG_INDEX_32I;
    int32_t* spill = nullptr;       // rows the short-row kernel hands to the general kernel
    unsigned long long* scan_status = nullptr;   // look-back scan: ticket + one word per tile
    bool use_short = false;         // dispatch the short-row kernel first
    bool use_row = true;            // short rows: k_row (false: the owner-round k_short)
    bool use_tile = false;          // wide-row path: (row, column tile) items
    bool lean = true;               // fp64 tiles may use the ordered-LDS kernels (k_tile_dn / k_tile_sp)
    bool lean32 = true;             // fp32 dense tiles may use the entry-run kernel (k_tile_dn<float>)
    int tws = 10;                   // log2 of the tile width
    int G = 1;                      // tiles per row
    int TR = 1;                     // tiles per wave task (a run of one row's tiles)
    int rgs = 0;                    // log2 of the tiles per record group (tile-major B's layout: RG
                                    // adjacent tiles' segments of a B row side by side)
    int twss = 10;                  // log2 of the symbolic tile width (>= tws, <= 16)
    bool sym_seg = false;           // symbolic tiles by the segment-walking kernel (long segments)
    bool counts_ready = false;      // a symbolic pass has completed (counts / offsets valid)
    unsigned long long* lb = nullptr;   // ALG1 single pass: per-row look-back status words
    void* ext = nullptr;            // ALG1 on k_row: every A entry's B row extent (RowExt)
    bool alg1_fused = false;        // C's arrays were written compact into tj/tx by one pass
    bool fused_failed = false;      // the single pass met a row it cannot take
    bool scaled_in_place = false;   // spg_numeric scaled the workspace result by alpha
    int64_t sym_spills = -1;        // rows the symbolic short-row pass spilled (-1 unknown)
    // ALG2/ALG3 on k_row: the count pass counts spilled rows itself and lists each chunk's
    // spills at p.spill + (chunk's first row), counted in cspill[c] (int32 in an int64 slot
    // after the 16 scalars); the numeric general kernel runs only for chunks with spills
    int64_t nspc = 0;
    int64_t* cspill = nullptr;
    std::vector<int64_t> chunk_spills;
    int64_t cap = 0;                // ALG1 single pass: entries tj/tx hold (an estimate)
    uint2* tidx = nullptr;          // B column-tile index, B.rows * G (start, end) pairs (a
                                    // temporary in the bitmap region, read before the symbolic pass)
    int32_t* tptr = nullptr;        // tile-major B: segment table, G * (B.rows + 1)
    uint32_t* sidx = nullptr;       // symbolic-tile starts inside each B row, B.rows * (Gs + 1)
    void* brec = nullptr;           // tile-major B: (column, value) records (numeric tile pass)
    uint16_t* bj16 = nullptr;       // B's columns modulo 65536 (symbolic tile pass)
    bool brec_built = false;      // whole records (columns + values) from B
    bool brec_cols = false;       // their column parts (spg_numeric_tiles fills the values)
    uint32_t* bitmap = nullptr;     // per-item column bitmaps (symbolic -> numeric)
    int64_t* item_cnt = nullptr;    // per-item counts, scanned in place into offsets
    bool tidx_built = false;
    unsigned list_grid = 16;        // blocks of the general kernel that takes its spills
    int symbolic_runs = 0;          // spg_symbolic may be called again (e.g. int32 -> int64)
    std::vector<int64_t> chunk_rows;   // ALG3 row boundaries (chunk c = [r[c], r[c+1]))
    std::vector<int64_t> chunk_nz;     // A entry offset of each boundary
};

// ----------------------------------------------------------------------------- helpers
namespace {

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

inline size_t vbytes(spg_dtype_t t) {
    return t == SPG_C_64F ? 16 : (t == SPG_R_64F || t == SPG_C_32F) ? 8 : 4;
}

// bytes of one tile-major B record of the tile path (column in tile + value, unpadded)
inline size_t brec_bytes(spg_dtype_t t) {
    return (SPG_REC10 && t == SPG_R_64F) ? 10 : (SPG_REC6 && t == SPG_R_32F) ? 6 : 4 + vbytes(t);
}

// Runs f(T{}) with T the C++ type of value type t.
// (SPG_ONLY_F64: fp64-only development builds for A/B timing, about 3x faster to compile;
// never shipped -- the other value types then return NOT_SUPPORTED.)
template <typename F>
spg_status_t dispatch_value(spg_dtype_t t, F&& f) {
    switch (t) {
#ifndef SPG_ONLY_F64
        case SPG_R_32F: return f(float(0));
        case SPG_C_32F: return f(cplx<float>(0));
        case SPG_C_64F: return f(cplx<double>(0));
#endif
        case SPG_R_64F: return f(double(0));
        default: break;
    }
    return SPG_STATUS_NOT_SUPPORTED;
}

// SPG_SHORT_KERNEL=short selects the owner-round k_short for short rows (A/B timing);
// the default is k_row.  Read once per process.
inline bool row_kernel_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SPG_SHORT_KERNEL");
        return !(e && std::strcmp(e, "short") == 0);
    }();
    return on;
}

// Tile numeric kernel variant (A/B timing builds only: `make HIPFLAGS+=-DSPG_TILE_RU=2` etc.;
// no environment variable can change what the shipped library computes).
//   SPG_TILE_RU     chunks per owner-round group (1, 2, or all in flight)
//   SPG_TILE_DENSE  0 turns the column-addressed accumulator off
//   SPG_TILE_TWS    log2 of a forced tile width (8..12; 0 = the planner's choice)
// The timing-only diagnostics (SPG_TILE_DIAG, results wrong) exist only in spgemm_tile.hpp
// builds that define it.
#ifndef SPG_TILE_RU
#define SPG_TILE_RU 1
#endif
#ifndef SPG_TILE_DENSE
#define SPG_TILE_DENSE 1
#endif
#ifndef SPG_TILE_TWS
#define SPG_TILE_TWS 0
#endif
//   SPG_TILE_LEAN   0 keeps the owner-round k_tile on dense tiles (A/B against k_tile_dn)
//   SPG_SYM8        symbolic tiles by the word-flattened walk (k_tile_sym8, default) instead of
//                   k_tile_sym (config 5: 20.1 -> 12.1 ms)
#ifndef SPG_SYM8
#define SPG_SYM8 1
#endif
//   SPG_SYM8_CW     waves per k_tile_sym8 task sharing one bitmap (1: k_tile_sym8, one wave per task)
#ifndef SPG_SYM8_CW
#define SPG_SYM8_CW 2
#endif
#ifndef SPG_TILE_LEAN
#define SPG_TILE_LEAN 1
#endif
//   SPG_SP_LEAN     0 keeps the owner-round k_tile on sparse tiles (A/B against k_tile_sp)
#ifndef SPG_SP_LEAN
#define SPG_SP_LEAN 1
#endif


struct TileVariant { int ru; bool dense; };
inline const TileVariant& tile_variant() {
    static const TileVariant v{SPG_TILE_RU, SPG_TILE_DENSE != 0};
    return v;
}

inline int64_t grid_for(int64_t rows, int per_block) { return (rows + per_block - 1) / per_block; }

inline int64_t scan_tiles(int64_t n) { return n > 0 ? (n + SCAN_TILE - 1) / SCAN_TILE : 1; }
// 64-row groups (ALG1 on k_row: one published prefix per group)
inline int64_t row_groups(int64_t n) { return (n + WAVE - 1) / WAVE; }

// Rows of the expected shape go to the short-row kernel first; the rest (and every row it
// rejects) to the general windowed kernels.  Only a scheduling choice: results are the
// same either way.
inline bool want_short(const spg_csr_t& A, const spg_csr_t& B) {
    if (B.cols > 32LL * ShortSmall::NW || A.rows == 0) return false;
    const double avgA = (double)A.nnz / (double)A.rows;
    const double avgB = B.rows > 0 ? (double)B.nnz / (double)B.rows : 0.0;
    return avgA <= 48.0 && avgA * avgB <= 400.0;
}

// Wide rows go to the tile path when their C rows are dense enough that a tile of up to
// 4096 columns holds a useful number of entries.  The tile width keeps the expected
// entries of a tile within TILE_CAP (or is at most TILE_CAP, which bounds them).
// `lean`: the fp64 ordered-LDS kernels (k_tile_dn / k_tile_sp) may run -- the build allows them
// and the handle's run-time check found the LDS ordering they rely on (spg_create)
inline bool want_tile(const spg_csr_t& A, const spg_csr_t& B, int& tws, int& G, bool lean) {
    if (A.rows == 0 || B.rows == 0 || B.cols == 0 || A.nnz == 0 || B.nnz == 0) return false;
    const double avgA = (double)A.nnz / (double)A.rows;
    const double avgB = (double)B.nnz / (double)B.rows;
    const double frac = 1.0 - std::exp(-avgA * avgB / (double)B.cols);   // expected C row density
    tws = 8;
    for (int t = 8; t <= 12; ++t) {
        const double tw = (double)(1 << t);
        if (tw <= TILE_CAP || frac * tw <= 0.95 * TILE_CAP) tws = t;
        if (tw >= (double)B.cols) break;
    }
    // fp64 C rows at least half dense and wide: dense tiles of 2048 columns (a 2048-slot
    // accumulator).  Half the items, half the segment-table lookups per product; config 4
    // measured 24.9 against 26.6 ms per product with 1024-column tiles.
    if (B.value_type == SPG_R_64F && lean && tws == 10 && frac >= 0.5 && B.cols >= 16384) tws = SPG_DN_WIDE_TWS;
    // fp64 C rows 10-24 % dense over >= 16384 columns: sparse tiles of 8192 columns (2048-slot
    // windows; half the items, A-row reads and segment-table lookups of 4096-column tiles;
    // config 5: 149.3 -> 124.8 ms per product)
    if (B.value_type == SPG_R_64F && lean && SPG_SP_LEAN && tws == 12 && frac >= 0.1 &&
        B.cols >= 16384 && frac * 8192.0 <= 0.95 * 2048)
        tws = 13;
    // (A/B timing builds only; at most 8192 columns: k_tile_sp<.., 2048> holds 256 bitmap words)
    if (SPG_TILE_TWS >= 8 && SPG_TILE_TWS <= 13) tws = SPG_TILE_TWS;
    if (frac * (double)(1 << tws) < 64.0) return false;
    // the tile-major B's segment table is int32 and its records are addressed with 32-bit
    // byte offsets
    if (B.nnz > 2147483647LL ||
        (double)(B.nnz + SENT_REGIONS * SENT_N) * (double)brec_bytes(B.value_type) >= 4294967296.0)
        return false;
    G = (int)((B.cols + (1 << tws) - 1) >> tws);
    return (double)A.rows * G < 2.0e9;
}

// grid of a tile kernel over `tasks` wave tasks: a multiple of 8 (XCD-aware block ids).  The
// kernels stride over their tasks, so the grid is capped: its work-item count must stay below
// 2^32 (the dispatch packet's grid size is 32-bit; 33.5M two-wave blocks failed to launch).
inline unsigned tile_grid(int64_t tasks, int wpb = TILE_WPB) {
    const int64_t cap = ((int64_t)1 << 31) / ((int64_t)wpb * WAVE);
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(grid_for(tasks, wpb), cap));
    return (unsigned)((nb + 7) / 8 * 8);
}
// grid of a cooperative tile kernel: one task per block of `wpb` waves (same caps)
inline unsigned coop_grid(int64_t tasks, int wpb) {
    const int64_t cap = ((int64_t)1 << 31) / ((int64_t)wpb * WAVE);
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(tasks, cap));
    return (unsigned)((nb + 7) / 8 * 8);
}

// symbolic tile: the narrowest width >= the numeric tile whose B segments (expected B row
// entries per tile) reach 64 entries -- long coalesced reads -- capped at 65536 columns
// and at the (pow2-rounded) row width.  When the widest symbolic tile (65536 columns or the
// whole row) holds segments of >= SEG_MIN entries, that width and the segment-walking
// symbolic kernel (k_tile_sym_seg) are used instead.
#ifndef SPG_SEG_MIN
#define SPG_SEG_MIN 128
#endif
constexpr double SEG_MIN = SPG_SEG_MIN;   // (config 5 segments of 65: 25.9 ms against 20.7 for k_tile_sym)
inline int sym_tile_log2(const spg_csr_t& B, int tws, bool* seg = nullptr) {
    const double avgB = B.rows > 0 ? (double)B.nnz / (double)B.rows : 0.0;
    int tmax = tws;
    while (tmax < 16 && ((int64_t)1 << tmax) < B.cols) ++tmax;
    const double seg_max = avgB * std::min(1.0, (double)((int64_t)1 << tmax) / (double)std::max<int64_t>(B.cols, 1));
    if (seg) *seg = seg_max >= SEG_MIN;
    if (seg_max >= SEG_MIN) return tmax;
    int t = tws;
    while (t < 16 && ((int64_t)1 << t) < B.cols && avgB * (double)((int64_t)1 << t) / (double)B.cols < 64.0) ++t;
    return std::max(tws, std::min(t, SPG_SYM_MAXLOG));
}


// C rows expected full (1 - exp(-avgA * avgB / N) >= 0.999, e.g. config 3 at density 0.1): the
// segment-walking symbolic kernel stops a task once its bitmap is full (a pure shortcut: the
// structure it writes is the same)
inline bool sym_full(const spg_plan_s& p) {
    if (p.A.rows <= 0 || p.B.rows <= 0 || p.B.cols <= 0) return false;
    const double avgA = (double)p.A.nnz / (double)p.A.rows, avgB = (double)p.B.nnz / (double)p.B.rows;
    return avgA * avgB / (double)p.B.cols >= 6.9;
}

// Makes the handle's device current for one entry point and restores the caller's device
// on exit (cuSPARSE leaves the current device alone; so does this library).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if ((err = hipGetDevice(&prev)) != hipSuccess) return;
        if (prev != dev) err = hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

spg_status_t hip_fail(spg_handle_t h, hipError_t e) {
    if (h) h->last_hip = (int)e;
    if (e == hipErrorOutOfMemory) return SPG_STATUS_ALLOC_FAILED;
    return SPG_STATUS_HIP_ERROR;
}

#define SPG_HIP(h, expr)                                  \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_fail((h), e_);   \
    } while (0)

#define SPG_LAUNCHED(h) SPG_HIP(h, hipGetLastError())

// The LDS ordering the lean fp64 tile kernels rely on, checked on this device:
// k_lds_order_check runs LDSCHK_TRIALS trials of two ds_add_f64 instructions from all 64 lanes
// into 4 slots with operands whose rounded sums depend on the order; the host replays them in
// (instruction, lane) order.  Any bit difference sets *ordered = false.
template <typename T>
hipError_t lds_order_check_t(bool* ordered) {
    constexpr int N = LDSCHK_TRIALS * 2 * WAVE;
    std::vector<T> v(N);
    std::vector<int> slot(N);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    auto next = [&] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (int i = 0; i < N; ++i) {
        const uint64_t r = next();
        const double m = 1.0 + (double)(r >> 11) * (1.0 / 9007199254740992.0);   // [1, 2)
        v[i] = (T)std::ldexp((r & 1) ? -m : m, (int)((r >> 1) % 81) - 40);
        slot[i] = (int)((r >> 8) & 3);
    }
    T *dv = nullptr, *dout = nullptr;
    int* ds = nullptr;
    hipError_t e = hipMalloc((void**)&dv, sizeof(T) * N);
    if (e == hipSuccess) e = hipMalloc((void**)&ds, sizeof(int) * N);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(T) * 4 * LDSCHK_TRIALS);
    if (e == hipSuccess) e = hipMemcpy(dv, v.data(), sizeof(T) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(ds, slot.data(), sizeof(int) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_lds_order_check<T>, dim3(1), dim3(WAVE), 0, 0, (const T*)dv, (const int*)ds, dout);
        e = hipGetLastError();
    }
    std::vector<T> got(4 * LDSCHK_TRIALS);
    if (e == hipSuccess) e = hipMemcpy(got.data(), dout, sizeof(T) * got.size(), hipMemcpyDeviceToHost);
    bool ok = e == hipSuccess;
    for (int t = 0; ok && t < LDSCHK_TRIALS; ++t) {
        T acc[4] = {(T)0, (T)0, (T)0, (T)0};
        for (int i = t * 2 * WAVE; i < (t + 1) * 2 * WAVE; ++i) acc[slot[i]] = acc[slot[i]] + v[i];
        ok = std::memcmp(acc, &got[4 * t], sizeof(acc)) == 0;
    }
    *ordered = ok;
    if (dv) (void)hipFree(dv);
    if (ds) (void)hipFree(ds);
    if (dout) (void)hipFree(dout);
    return e;
}
// both widths, each its own flag: ds_add_f64 (the fp64 / complex128 lean kernels) and ds_add_f32
// (the fp32 runs' third-and-later entries, k_tile_dn<float, ..>) -- a device failing only the
// f32 check keeps the fp64 kernels
hipError_t lds_order_check(bool* o64, bool* o32) {
    *o64 = *o32 = false;
    hipError_t e = lds_order_check_t<double>(o64);
    if (e == hipSuccess) e = lds_order_check_t<float>(o32);
    return e;
}

hipEvent_t take_event(spg_handle_t h) {
    if (!h->pool.empty()) {
        hipEvent_t e = h->pool.back();
        h->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Brackets the kernel launches of one phase with events when timing is enabled.
struct PhaseTimer {
    spg_handle_t h;
    int phase;
    hipEvent_t a = nullptr;
    PhaseTimer(spg_handle_t h_, int phase_) : h(h_), phase(phase_) {
        if (h->timing && (a = take_event(h))) (void)hipEventRecord(a, h->stream);
    }
    ~PhaseTimer() {
        if (!a) return;
        hipEvent_t b = take_event(h);
        if (!b) { h->pool.push_back(a); return; }
        (void)hipEventRecord(b, h->stream);
        h->pending.push_back({phase, a, b});
    }
};

// Device time of ONE kernel launch (the numeric phases, the roofline's kernel): the events
// go into the launch's own dispatch packet (hipExtLaunchKernelGGL), so the interval is the
// kernel's run time; hipEventRecord markers around a launch add gaps of their own (3-4 us
// on the 28 us numeric pass of config 2).  Null events (timing off) record nothing.
struct KernelTimer {
    spg_handle_t h;
    int phase;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(spg_handle_t h_, int phase_) : h(h_), phase(phase_) {
        if (!h->timing || !(a = take_event(h))) return;
        if (!(b = take_event(h))) { h->pool.push_back(a); a = nullptr; }
    }
    ~KernelTimer() {
        if (a && b) h->pending.push_back({phase, a, b});
    }
};

// A launch timed by KernelTimer (every kernel of the timed phases: the phase time is the
// sum of its kernels' device times; marker events around launches drift once ext-launch
// events are on the stream).
template <typename K, typename... Args>
inline void timed_launch(spg_handle_t h, int phase, K kernel, dim3 grid, dim3 block, Args... args) {
    KernelTimer kt(h, phase);
    hipExtLaunchKernelGGL(kernel, grid, block, 0, h->stream, kt.a, kt.b, 0, args...);
}

spg_status_t check_csr(const spg_csr_t* M) {
    if (!M) return SPG_STATUS_INVALID_VALUE;
    if (M->rows < 0 || M->cols < 0 || M->nnz < 0) return SPG_STATUS_INVALID_VALUE;
    if (M->cols > 2147483647LL) return SPG_STATUS_NOT_SUPPORTED;   // int32 column indices
    if (M->indptr_type != SPG_INDEX_32I && M->indptr_type != SPG_INDEX_64I)
        return SPG_STATUS_INVALID_VALUE;
    if (M->value_type != SPG_R_32F && M->value_type != SPG_R_64F && M->value_type != SPG_C_32F &&
        M->value_type != SPG_C_64F)
        return SPG_STATUS_NOT_SUPPORTED;
    if (M->indptr_type == SPG_INDEX_32I && M->nnz > 2147483647LL) return SPG_STATUS_INVALID_VALUE;
    if (!M->indptr && M->rows >= 0) return SPG_STATUS_INVALID_VALUE;
    if (M->nnz > 0 && (!M->indices || !M->values)) return SPG_STATUS_INVALID_VALUE;
    return SPG_STATUS_SUCCESS;
}

spg_status_t ensure_scratch(spg_handle_t h, size_t bytes) {
    if (h->scratch_bytes >= bytes) return SPG_STATUS_SUCCESS;
    if (h->scratch) {
        SPG_HIP(h, hipStreamSynchronize(h->stream));
        SPG_HIP(h, hipFree(h->scratch));
        h->scratch = nullptr;
        h->scratch_bytes = 0;
    }
    SPG_HIP(h, hipMalloc(&h->scratch, bytes));
    h->scratch_bytes = bytes;
    return SPG_STATUS_SUCCESS;
}

// Product prefix of every row into `pref` (rows + 1 int64) and its total into scal[0].
// `status` (tiles + 1 words) must be zero: plans zero theirs once when they are built
template <typename OUT, typename IN = int64_t>
spg_status_t launch_scan(spg_handle_t h, int64_t n, const IN* in, OUT* out,
                         unsigned long long* status, int64_t* scal, bool zero_status,
                         int32_t* move_cnt = nullptr, int64_t* move_dst = nullptr,
                         int64_t* host_mirror = nullptr, int64_t mirror_gen = 0, int mirror_n = 0,
                         const int64_t* seed = nullptr) {
    const int64_t tiles = scan_tiles(n);
    if (zero_status)
        SPG_HIP(h, hipMemsetAsync(status, 0, sizeof(unsigned long long) * (size_t)(tiles + 1), h->stream));
    // (the handle's wait bound: SPG_LB_SPIN_TICKS=0 sends every look-back of an out-of-place
    // scan down its direct path, for the tests; in-place scans always wait, k_scan_lb)
    timed_launch(h, SPG_PHASE_SCAN, k_scan_lb<OUT, IN>, dim3((unsigned)tiles), dim3(BLOCK), n, in, out, status, scal,
                 move_cnt, move_dst, host_mirror, mirror_gen, mirror_n, seed, h->lb_spin);
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

template <typename IP>
spg_status_t launch_products(spg_handle_t h, const spg_csr_t& A, const spg_csr_t& B,
                             int64_t* cnt, int64_t* pref, int64_t* scal,
                             unsigned long long* status, bool zero_status) {
    const int64_t rows = A.rows;
    if (rows > 0) {
        PhaseTimer pt(h, SPG_PHASE_PRODUCTS);
        hipLaunchKernelGGL(k_row_products<IP>, dim3((unsigned)grid_for(rows, WPB)), dim3(BLOCK), 0,
                           h->stream, rows, (const IP*)A.indptr, (const int32_t*)A.indices,
                           (const IP*)B.indptr, cnt);
        SPG_LAUNCHED(h);
    }
    return launch_scan<int64_t>(h, rows, cnt, pref, status, scal, zero_status);
}

spg_status_t products_prefix(spg_handle_t h, const spg_csr_t& A, const spg_csr_t& B,
                             int64_t* cnt, int64_t* pref, int64_t* scal,
                             unsigned long long* status, bool zero_status = true) {
    return A.indptr_type == SPG_INDEX_64I ? launch_products<int64_t>(h, A, B, cnt, pref, scal, status, zero_status)
                                          : launch_products<int32_t>(h, A, B, cnt, pref, scal, status, zero_status);
}

spg_status_t read_scalars(spg_handle_t h, const int64_t* dev, int n, int64_t* out);

// P alone (no per-row prefix): one flat pass over A's entries into handle scratch
spg_status_t products_total(spg_handle_t h, const spg_csr_t& A, const spg_csr_t& B, int64_t* P) {
    spg_status_t st = ensure_scratch(h, 256);
    if (st) return st;
    unsigned long long* acc = (unsigned long long*)h->scratch;
    SPG_HIP(h, hipMemsetAsync(acc, 0, sizeof(unsigned long long), h->stream));
    if (A.nnz > 0) {
        PhaseTimer pt(h, SPG_PHASE_PRODUCTS);
        const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(A.nnz, 4 * BLOCK), 256));
        if (A.indptr_type == SPG_INDEX_64I)
            hipLaunchKernelGGL(k_products_total<int64_t>, dim3(grid), dim3(BLOCK), 0, h->stream, A.nnz,
                               (const int32_t*)A.indices, (const int64_t*)B.indptr, acc);
        else
            hipLaunchKernelGGL(k_products_total<int32_t>, dim3(grid), dim3(BLOCK), 0, h->stream, A.nnz,
                               (const int32_t*)A.indices, (const int32_t*)B.indptr, acc);
        SPG_LAUNCHED(h);
    }
    return read_scalars(h, (const int64_t*)acc, 1, P);
}

// handle scratch for plan-time product prefixes: cnt[rows] | pref[rows+1] | scal[16] | status
struct ScratchView {
    int64_t* cnt;
    int64_t* pref;
    int64_t* scal;
    unsigned long long* status;
};

spg_status_t scratch_for_products(spg_handle_t h, int64_t rows, ScratchView& v) {
    const size_t words = 2 * (size_t)rows + 1 + 16 + (size_t)scan_tiles(rows) + 1;
    spg_status_t st = ensure_scratch(h, sizeof(int64_t) * words);
    if (st) return st;
    v.cnt = (int64_t*)h->scratch;
    v.pref = v.cnt + rows;
    v.scal = v.pref + rows + 1;
    v.status = (unsigned long long*)(v.scal + 16);
    return SPG_STATUS_SUCCESS;
}

// Waits for the handle's stream (polling hipStreamQuery measured slower on the box).
hipError_t stream_wait(spg_handle_t h) { return hipStreamSynchronize(h->stream); }

// Waits until the scan of generation h->mirror_gen has written its scalars to the pinned
// buffer.  The numeric pass behind it stays queued on the stream: the call returns while it
// runs (the results are stream-ordered, like every other output of the library).  A stream
// that drains without the generation arriving, or reports an error, fails the call.
spg_status_t wait_mirror(spg_handle_t h) {
    const volatile int64_t* gen = (const volatile int64_t*)h->pinned + MIRROR_GEN_WORD;
    for (unsigned spin = 1; *gen != h->mirror_gen; ++spin) {
        if ((spin & 1023) == 0) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e == hipSuccess) {
                if (*gen == h->mirror_gen) break;
                return SPG_STATUS_EXECUTION_FAILED;
            }
            if (e != hipErrorNotReady) SPG_HIP(h, e);
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return SPG_STATUS_SUCCESS;
}

spg_status_t read_scalars(spg_handle_t h, const int64_t* dev, int n, int64_t* out) {
    if (n > MIRROR_GEN_WORD) return SPG_STATUS_INTERNAL_ERROR;   // never reaches the generation word
    SPG_HIP(h, hipMemcpyAsync(h->pinned, dev, sizeof(int64_t) * n, hipMemcpyDeviceToHost, h->stream));
    SPG_HIP(h, stream_wait(h));
    for (int i = 0; i < n; ++i) out[i] = h->pinned[i];
    return SPG_STATUS_SUCCESS;
}

struct Layout {
    size_t scalars = 0, row_cnt = 0, seg = 0, spill = 0, status = 0, ub = 0, tj = 0, tx = 0;
    size_t tptr = 0, sidx = 0, items = 0, bitmap = 0, brec = 0, bj16 = 0, ext = 0, total = 0;
};

// Tile path row chunks: ALG3's chunks (items and bitmaps are sized by the largest one and
// reused chunk by chunk -- the working set ALG3 caps), otherwise all rows in one.
inline int64_t tile_chunks(const spg_plan_s& p) {
    return p.alg == SPG_ALG3 && p.chunk_rows.size() > 1 ? (int64_t)p.chunk_rows.size() - 1 : 1;
}
inline int64_t tile_chunk_r0(const spg_plan_s& p, int64_t c) { return tile_chunks(p) > 1 ? p.chunk_rows[(size_t)c] : 0; }
inline int64_t tile_chunk_r1(const spg_plan_s& p, int64_t c) {
    return tile_chunks(p) > 1 ? p.chunk_rows[(size_t)c + 1] : p.A.rows;
}
inline int64_t tile_rows_max(const spg_plan_s& p) {
    int64_t mx = 0;
    for (int64_t c = 0; c < tile_chunks(p); ++c) mx = std::max(mx, tile_chunk_r1(p, c) - tile_chunk_r0(p, c));
    return mx;
}
inline int64_t tile_items(const spg_plan_s& p) { return p.use_tile ? tile_rows_max(p) * p.G : 0; }
// Dense numeric tiles (one accumulator window per tile) take an item's structure from the
// accumulation itself: no symbolic bitmaps, and every item's 8-byte offset is kept (all
// rows, not one chunk's), so ALG3's numeric phase does not recompute its chunks' counts.
inline bool tile_dense(const spg_plan_s& p) {
    const int cap = (p.A.value_type == SPG_R_64F && p.lean) ? DN_TW_MAX : TILE_CAP;   // (k_tile_dn<.., 2048>)
    return p.use_tile && (1 << p.tws) <= cap && tile_variant().dense;
}
inline int64_t tile_item_slots(const spg_plan_s& p) { return tile_dense(p) ? p.A.rows * p.G : tile_items(p); }
// item counts / offsets of chunk c (dense tiles: every chunk's stay, at its rows' place)
inline int64_t* tile_chunk_items(const spg_plan_s& p, int64_t c) {
    return tile_dense(p) ? p.item_cnt + tile_chunk_r0(p, c) * p.G : p.item_cnt;
}
inline int sym_tiles(const spg_plan_s& p) { const int R = 1 << (p.twss - p.tws); return (p.G + R - 1) / R; }
// record groups of the tile-major B: Gq groups of RG = 1 << rgs tiles (the last padded to RG)
inline int64_t rec_groups(const spg_plan_s& p) { return ((int64_t)p.G + (1 << p.rgs) - 1) >> p.rgs; }
inline int64_t tiles_padded(const spg_plan_s& p) { return rec_groups(p) << p.rgs; }
inline int64_t group_words(const spg_plan_s& p) { return (p.B.rows << p.rgs) + 1; }   // one group's table
inline int64_t bt_entries(const spg_plan_s& p) { return p.use_tile ? rec_groups(p) * group_words(p) : 0; }
// fp32 dense tiles take k_tile_dn<float, .., 1024> (plain read-add-write per A entry's run of a
// chunk) when a tile's expected B segment holds >= SPG_F32_RUN_MIN entries: chunks then hold one
// or two entries' runs (config 3 at density 0.1: 102-entry segments); shorter segments put many
// entries in a chunk and keep k_tile's owner rounds.  SPG_F32_RUNS=0 (read per plan: a
// schedule-only switch for A/B timing and the tests) keeps k_tile.
#ifndef SPG_F32_RUN_MIN
#define SPG_F32_RUN_MIN 48
#endif
inline bool fp32_runs(const spg_plan_s& p) {
    if (!p.lean32 || p.A.value_type != SPG_R_32F || p.B.cols <= 0 || p.B.rows <= 0 || (1 << p.tws) > 1024) return false;
    const char* e = std::getenv("SPG_F32_RUNS");
    if (e && std::strcmp(e, "0") == 0) return false;
    const double seg = (double)p.B.nnz / (double)p.B.rows * (double)(1 << p.tws) / (double)p.B.cols;
    return seg >= SPG_F32_RUN_MIN;
}
// fp64 8192-column sparse tiles (config 5's shape) run in cooperative record groups of
// 1 << SPG_SP_RGS tiles (k_tile_sp<.., RG>), on a persistent grid of 8 / RG blocks per CU.
// Measured on config 5 (round 5, numeric ms per product): RG 1 97.6 (511 GB of fabric reads per
// launch); RG 4 with one block per item 103 (361 GB: the block's waves idle until its slowest
// item ends, and a new block needs a whole block's LDS); RG 4 persistent 92.7 (367 GB), RG 8
// persistent 91.8 (301 GB), RG 2 persistent 101.3; RG 1 persistent 118.5 (one-wave blocks
// balance best dispatched one item each).  On the final kernels (saddr record loads), alternated
// on one box: RG 8 89.7-89.8 against RG 4 91.0-91.3 (abtest/r05_call24.sh) -- RG 8, one 8-wave
// block per CU (159.6 KiB of LDS).  SPG_SP_RGS=0 builds keep RG = 1.
#ifndef SPG_SP_RGS
#define SPG_SP_RGS 3
#endif
// (SPG_SP_RECORD_GROUP=1, read per plan: a schedule-only switch to the one-wave kernel over
// plain tile-major records, for A/B timing and for the tests; results are identical)
// (SPG_DN_RGS = 1, A/B builds: fp64 2048-column dense tiles in record groups of 2, one per
// 2-wave block of k_tile_dn<.., RG = 2> on a persistent grid; config 4 numeric 22.4 ms against
// 19.1 ms for independent items, round 5)
#ifndef SPG_DN_RGS
#define SPG_DN_RGS 0
#endif
#ifndef SPG_DN_RG_PERSIST
#define SPG_DN_RG_PERSIST 1
#endif
inline int record_group_log2(const spg_plan_s& p) {
    if (SPG_DN_RGS > 0 && p.use_tile && tile_dense(p) && p.lean && p.A.value_type == SPG_R_64F && p.tws == 11)
        return SPG_DN_RGS;
    if (!p.use_tile || tile_dense(p) || !p.lean || !SPG_SP_LEAN) return 0;
    if (p.A.value_type != SPG_R_64F || p.tws != 13) return 0;
    const char* e = std::getenv("SPG_SP_RECORD_GROUP");
    if (e && std::strcmp(e, "1") == 0) return 0;
    return SPG_SP_RGS;
}

// ALG1 runs as one fused pass (k_short SHORT_NUMLB) when the short-row kernel takes the shape
inline bool fused_alg1(const spg_plan_s& p) {
    return p.alg == SPG_ALG1 && p.use_short && !p.use_tile && p.A.rows <= (1LL << 24);
}

// status words: products scan | row-pointer scan | item scan + segment-table scan (tile path)
inline size_t status_words(const spg_plan_s& p) {
    return 2 * (size_t)(scan_tiles(p.A.rows) + 1) +
           (p.use_tile ? (size_t)scan_tiles(tile_items(p)) + 1 + (size_t)scan_tiles(bt_entries(p)) + 1 : 0) +
           (fused_alg1(p) ? (size_t)std::max<int64_t>(grid_for(p.A.rows, ShortSmall::WPB), row_groups(p.A.rows)) + 1 : 0);
}
inline unsigned long long* item_scan_status(const spg_plan_s& p) {
    return p.scan_status + 2 * (scan_tiles(p.A.rows) + 1);
}
inline unsigned long long* bt_scan_status(const spg_plan_s& p) {
    return item_scan_status(p) + scan_tiles(tile_items(p)) + 1;
}

Layout make_layout(const spg_plan_s& p) {
    Layout L;
    size_t off = 0;
    L.scalars = off; off = align_up(off + (16 + (size_t)p.nspc) * sizeof(int64_t));
    L.status = off;  off = align_up(off + sizeof(unsigned long long) * status_words(p));
    L.row_cnt = off; off = align_up(off + sizeof(int64_t) * (size_t)(p.A.rows + 1));
    L.seg = off;     off = align_up(off + sizeof(uint32_t) * 2 * (size_t)std::max<int64_t>(p.seg_len, 1));
    L.spill = off;   off = align_up(off + sizeof(int32_t) * 2 * (size_t)std::max<int64_t>(p.A.rows, 1));
    if (p.use_tile) {
        L.tptr = off;  off = align_up(off + sizeof(int32_t) * (size_t)(bt_entries(p) + 1));
        L.sidx = off;  off = align_up(off + sizeof(uint32_t) * (size_t)p.B.rows * (size_t)(sym_tiles(p) + 1));
        // (B's records, then the lean kernels' sentinel records)
        L.brec = off;  off = align_up(off + brec_bytes(p.A.value_type) * (size_t)(p.B.nnz + SENT_REGIONS * SENT_N));
        L.items = off; off = align_up(off + sizeof(int64_t) * (size_t)(tile_item_slots(p) + 1));
        // B's column indices modulo 65536 (the symbolic pass's columns: a symbolic tile never
        // crosses a 65536-aligned block)
        L.bj16 = off;  off = align_up(off + sizeof(uint16_t) * (size_t)(p.B.nnz + 8));   // (+8: whole 16-byte loads)
        // item bitmaps; before the first symbolic pass the region holds the row-major
        // boundary index the tile-major B is built from
        const size_t bm = tile_dense(p) ? 0 : sizeof(uint32_t) * (size_t)tile_items(p) * (size_t)((1 << p.tws) >> 5);
        const size_t ti = sizeof(uint2) * (size_t)p.B.rows * (size_t)tiles_padded(p);
        L.bitmap = off; off = align_up(off + std::max(bm, ti));
    }
    if (p.alg == SPG_ALG1 && !p.use_tile) {
        // single pass: C itself, `cap` entries (an estimate); upper-bound path: P entries
        const int64_t n = fused_alg1(p) ? p.cap : p.P;
        if (!fused_alg1(p)) { L.ub = off; off = align_up(off + sizeof(int64_t) * (size_t)(p.A.rows + 1)); }
        if (fused_alg1(p) && p.use_row) {
            const size_t eb = p.A.indptr_type == SPG_INDEX_64I ? sizeof(RowExt<int64_t>) : sizeof(RowExt<int32_t>);
            L.ext = off; off = align_up(off + eb * (size_t)std::max<int64_t>(p.A.nnz, 1));
        }
        L.tj = off; off = align_up(off + sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1));
        L.tx = off; off = align_up(off + vbytes(p.A.value_type) * (size_t)std::max<int64_t>(n, 1));
    }
    L.total = off;
    return L;
}

void carve(spg_plan_s& p, const Layout& L) {
    p.scalars = (int64_t*)(p.ws + L.scalars);
    p.cspill = p.nspc > 0 ? p.scalars + 16 : nullptr;
    p.row_cnt = (int64_t*)(p.ws + L.row_cnt);
    p.seg = (uint32_t*)(p.ws + L.seg);
    p.spill = (int32_t*)(p.ws + L.spill);
    p.scan_status = (unsigned long long*)(p.ws + L.status);
    if (fused_alg1(p)) p.lb = p.scan_status + 2 * (scan_tiles(p.A.rows) + 1);
    if (p.use_tile) {
        p.tptr = (int32_t*)(p.ws + L.tptr);
        p.sidx = (uint32_t*)(p.ws + L.sidx);
        p.tidx = (uint2*)(p.ws + L.bitmap);
        p.brec = (void*)(p.ws + L.brec);
        p.bj16 = (uint16_t*)(p.ws + L.bj16);
        p.item_cnt = (int64_t*)(p.ws + L.items);
        p.bitmap = (uint32_t*)(p.ws + L.bitmap);
    }
    if (p.alg == SPG_ALG1 && !p.use_tile) {
        if (!fused_alg1(p)) p.ub = (int64_t*)(p.ws + L.ub);
        if (fused_alg1(p) && p.use_row) p.ext = (void*)(p.ws + L.ext);
        p.tj = (int32_t*)(p.ws + L.tj);
        p.tx = (void*)(p.ws + L.tx);
    }
}

// ALG3: cut rows into chunks of at most max(cf * P, largest row) products.
spg_status_t plan_chunks(spg_handle_t h, spg_plan_s& p) {
    const int64_t rows = p.A.rows;
    p.chunk_rows.assign({0, rows});
    p.chunk_nz.assign({0, p.A.nnz});
    p.seg_len = p.A.nnz;
    if (rows == 0) return SPG_STATUS_SUCCESS;
    ScratchView sv;
    spg_status_t st = scratch_for_products(h, rows, sv);
    if (st) return st;
    int64_t* pref = sv.pref;
    if ((st = products_prefix(h, p.A, p.B, sv.cnt, sv.pref, sv.scal, sv.status))) return st;
    std::vector<int64_t> hp((size_t)rows + 1), ha((size_t)rows + 1);
    SPG_HIP(h, hipMemcpyAsync(hp.data(), pref, sizeof(int64_t) * (rows + 1), hipMemcpyDeviceToHost, h->stream));
    if (p.A.indptr_type == SPG_INDEX_64I) {
        SPG_HIP(h, hipMemcpyAsync(ha.data(), p.A.indptr, sizeof(int64_t) * (rows + 1),
                                  hipMemcpyDeviceToHost, h->stream));
        SPG_HIP(h, hipStreamSynchronize(h->stream));
    } else {
        std::vector<int32_t> t((size_t)rows + 1);
        SPG_HIP(h, hipMemcpyAsync(t.data(), p.A.indptr, sizeof(int32_t) * (rows + 1),
                                  hipMemcpyDeviceToHost, h->stream));
        SPG_HIP(h, hipStreamSynchronize(h->stream));
        for (int64_t i = 0; i <= rows; ++i) ha[(size_t)i] = t[(size_t)i];
    }
    p.P = hp[(size_t)rows];
    const int64_t cap = std::max<int64_t>(1, (int64_t)std::ceil((double)p.cf * (double)p.P));
    // n chunks of about equal products, n from ceil(P / cap) up: cut k lands on the row end
    // nearest k*P/n such that chunk k stays within the cap and what is left still fits the
    // remaining chunks.  Row ends rarely fall on k*P/n exactly, so chunk_fraction 0.2 gives
    // six chunks of 16.7 % (a greedy fill to the cap gives 5 x 19.99 % + one tiny chunk).
    // Rows longer than the slack fall back to the greedy fill (at least one row per chunk).
    auto last_le = [&](int64_t r, int64_t v) {   // last row end e > r with pref[e] <= v (or r)
        return (int64_t)(std::upper_bound(hp.begin() + r + 1, hp.end(), v) - hp.begin()) - 1;
    };
    int64_t n = std::max<int64_t>(1, (p.P + cap - 1) / cap);
    for (int attempt = 0; attempt < 3; ++attempt, ++n) {
        p.chunk_rows.assign(1, 0);
        p.chunk_nz.assign(1, ha[0]);
        int64_t r = 0;
        for (int64_t k = 1; r < rows; ++k) {
            int64_t e = last_le(r, hp[(size_t)r] + cap);   // the greedy bound
            if (k < n && e < rows) {
                const int64_t target = (int64_t)((long double)p.P * (long double)k / (long double)n);
                const int64_t need = p.P - (n - k) * cap;   // pref[e] >= need: the rest fits
                int64_t b = last_le(r, target);
                if (b + 1 <= e && hp[(size_t)b + 1] - target < target - hp[(size_t)b]) ++b;
                if (hp[(size_t)b] < need)
                    b = std::min(e, (int64_t)(std::lower_bound(hp.begin() + r + 1, hp.end(), need) - hp.begin()));
                e = std::min(e, b);
            }
            if (e <= r) e = r + 1;
            p.chunk_rows.push_back(e);
            p.chunk_nz.push_back(ha[(size_t)e]);
            r = e;
        }
        if ((int64_t)p.chunk_rows.size() - 1 <= n) break;
    }
    int64_t mx = 0;
    for (size_t c = 0; c + 1 < p.chunk_nz.size(); ++c)
        mx = std::max(mx, p.chunk_nz[c + 1] - p.chunk_nz[c]);
    p.seg_len = mx;
    return SPG_STATUS_SUCCESS;
}

// --------------------------------------------------------------------- typed launchers
// Spill chain of the short-row path: small rows -> list 1 -> medium rows -> list 2 ->
// general windowed kernel.  Counters live in scalars[4] (int32 x2).
// scalars[4]: two int32 spill counters of the symbolic phase; scalars[5]: of the numeric
// phase.  The whole control block (scalars + scan status words) is zeroed once per plan.
inline int32_t* spill_counts(spg_plan_s& p, bool numeric) {
    return (int32_t*)(p.scalars + (numeric ? 5 : 4));
}

template <typename IP>
spg_status_t run_symbolic_rows(spg_handle_t h, spg_plan_s& p, int64_t r0, int64_t r1, int64_t nz0, int chunk = 0) {
    const int64_t n = r1 - r0;
    if (n <= 0) return SPG_STATUS_SUCCESS;
    const IP* Ap = (const IP*)p.A.indptr;
    const IP* Bp = (const IP*)p.B.indptr;
    const int32_t* Aj = (const int32_t*)p.A.indices;
    const int32_t* Bj = (const int32_t*)p.B.indices;
    if (p.use_tile) {
        return SPG_STATUS_INTERNAL_ERROR;   // the tile path runs through tile_symbolic
    } else if (p.use_short && p.nspc > 0) {
        // k_row counts every row (spills by the chunked loop) and lists this chunk's spills
        timed_launch(h, SPG_PHASE_SYMBOLIC, k_row<double, IP, int64_t, ROW_SYM, RowSmall>,
                           dim3((unsigned)grid_for(n, RowSmall::WPB * row_pair<ROW_SYM>())), dim3(RowSmall::WPB * WAVE),
                           r0, n, p.B.cols, Ap, Aj, (const double*)nullptr, Bp, Bj,
                           (const double*)nullptr, (const int64_t*)nullptr, (int32_t*)nullptr, (double*)nullptr,
                           1.0, p.row_cnt, p.spill + r0, (int32_t*)(p.cspill + chunk), (int)ROW_COUNT_ALL,
                           (int64_t)0, (const int64_t*)nullptr, (unsigned long long*)nullptr, (int64_t)0,
                           (RowExt<IP>*)nullptr, RowScan<int64_t>{});
    } else if (p.use_short) {
        int32_t* cnt = spill_counts(p, false);
        int32_t* l1 = p.spill;
        {
            PhaseTimer pt(h, SPG_PHASE_SYMBOLIC);
            if (p.use_row)
                hipLaunchKernelGGL((k_row<double, IP, int64_t, ROW_SYM, RowSmall>),
                                   dim3((unsigned)grid_for(n, RowSmall::WPB * row_pair<ROW_SYM>())), dim3(RowSmall::WPB * WAVE), 0,
                                   h->stream, r0, n, p.B.cols, Ap, Aj, (const double*)nullptr, Bp, Bj,
                                   (const double*)nullptr, (const int64_t*)nullptr, (int32_t*)nullptr,
                                   (double*)nullptr, 1.0, p.row_cnt, l1, cnt, 0, (int64_t)0,
                                   (const int64_t*)nullptr, (unsigned long long*)nullptr, (int64_t)0,
                                   (RowExt<IP>*)nullptr, RowScan<int64_t>{});
            else
                hipLaunchKernelGGL((k_short<double, IP, int64_t, SHORT_SYM, ShortSmall>),
                                   dim3((unsigned)grid_for(n, ShortSmall::WPB)), dim3(ShortSmall::WPB * WAVE), 0,
                                   h->stream, r0, n, p.B.cols, Ap, Aj, (const double*)nullptr, Bp, Bj,
                                   (const double*)nullptr, (const int64_t*)nullptr, (int32_t*)nullptr,
                                   (double*)nullptr, 1.0, p.row_cnt, l1, cnt, (const int32_t*)nullptr,
                                   (const int32_t*)nullptr, (unsigned long long*)nullptr, (int64_t*)nullptr,
                                   (int64_t*)nullptr, (int64_t)0);
            SPG_LAUNCHED(h);
        }
        PhaseTimer ps(h, SPG_PHASE_SPILL);
        hipLaunchKernelGGL(k_symbolic<IP>, dim3(p.list_grid), dim3(BLOCK), 0, h->stream, r0, n,
                           p.B.cols, Ap, Aj, Bp, Bj, p.row_cnt, p.seg, nz0, (const int32_t*)l1,
                           (const int32_t*)cnt);
    } else {
        PhaseTimer pt(h, SPG_PHASE_SYMBOLIC);
        hipLaunchKernelGGL(k_symbolic<IP>, dim3((unsigned)grid_for(n, WPB)), dim3(BLOCK), 0, h->stream,
                           r0, n, p.B.cols, Ap, Aj, Bp, Bj, p.row_cnt, p.seg, nz0,
                           (const int32_t*)nullptr, (const int32_t*)nullptr);
    }
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

template <typename T, typename IP, typename OFF, bool UB>
spg_status_t run_numeric_rows(spg_handle_t h, spg_plan_s& p, int64_t r0, int64_t r1, int64_t nz0,
                              const OFF* off, int32_t* cj, T* cx, T alpha, int chunk = 0) {
    const int64_t n = r1 - r0;
    if (n <= 0) return SPG_STATUS_SUCCESS;
    const IP* Ap = (const IP*)p.A.indptr;
    const IP* Bp = (const IP*)p.B.indptr;
    const int32_t* Aj = (const int32_t*)p.A.indices;
    const int32_t* Bj = (const int32_t*)p.B.indices;
    const T* Ax = (const T*)p.A.values;
    const T* Bx = (const T*)p.B.values;
    constexpr int MODE = UB ? SHORT_NUMUB : SHORT_NUM;
    if (p.use_tile) {
        return SPG_STATUS_INTERNAL_ERROR;   // the tile path runs through tile_numeric
    } else if (p.use_short && p.nspc > 0 && !UB) {
        {
            KernelTimer kt(h, SPG_PHASE_NUMERIC);
            hipExtLaunchKernelGGL((k_row<T, IP, OFF, ROW_NUM, RowSmall>), dim3((unsigned)grid_for(n, RowSmall::WPB * row_pair<ROW_NUM>())),
                                  dim3(RowSmall::WPB * WAVE), 0, h->stream, kt.a, kt.b, 0, r0, n, p.B.cols, Ap, Aj, Ax,
                                  Bp, Bj, Bx, off, cj, cx, alpha, p.row_cnt, p.spill + r0, (int32_t*)(p.cspill + chunk),
                                  (int)ROW_LISTED, (int64_t)0, (const int64_t*)nullptr,
                                  (unsigned long long*)nullptr, (int64_t)0, (RowExt<IP>*)nullptr, RowScan<OFF>{});
            SPG_LAUNCHED(h);
        }
        // the general kernel only for a chunk whose count pass listed rows
        if ((size_t)chunk < p.chunk_spills.size() && p.chunk_spills[(size_t)chunk] == 0) return SPG_STATUS_SUCCESS;
        PhaseTimer ps(h, SPG_PHASE_SPILL);
        hipLaunchKernelGGL((k_numeric<T, IP, OFF, UB>), dim3(p.list_grid), dim3(BLOCK), 0, h->stream,
                           r0, n, p.B.cols, Ap, Aj, Ax, Bp, Bj, Bx, off, cj, cx, alpha, p.row_cnt,
                           p.seg, nz0, p.seg_len, (const int32_t*)(p.spill + r0),
                           (const int32_t*)(p.cspill + chunk));
    } else if (p.use_short) {
        int32_t* cnt = spill_counts(p, true);
        int32_t* l1 = p.spill;
        {
            PhaseTimer pt(h, SPG_PHASE_NUMERIC);
            if (p.use_row && !UB)
                hipLaunchKernelGGL((k_row<T, IP, OFF, ROW_NUM, RowSmall>), dim3((unsigned)grid_for(n, RowSmall::WPB * row_pair<ROW_NUM>())),
                                   dim3(RowSmall::WPB * WAVE), 0, h->stream, r0, n, p.B.cols, Ap, Aj, Ax, Bp, Bj,
                                   Bx, off, cj, cx, alpha, p.row_cnt, l1, cnt, 0, (int64_t)0,
                                   (const int64_t*)nullptr, (unsigned long long*)nullptr, (int64_t)0,
                                   (RowExt<IP>*)nullptr, RowScan<OFF>{});
            else
                hipLaunchKernelGGL((k_short<T, IP, OFF, MODE, ShortSmall>), dim3((unsigned)grid_for(n, ShortSmall::WPB)),
                                   dim3(ShortSmall::WPB * WAVE), 0, h->stream, r0, n, p.B.cols, Ap, Aj, Ax, Bp, Bj,
                                   Bx, off, cj, cx, alpha, p.row_cnt, l1, cnt, (const int32_t*)nullptr,
                                   (const int32_t*)nullptr, (unsigned long long*)nullptr, (OFF*)nullptr,
                                   (int64_t*)nullptr, (int64_t)0);
            SPG_LAUNCHED(h);
        }
        if (p.sym_spills == 0) return SPG_STATUS_SUCCESS;
        PhaseTimer ps(h, SPG_PHASE_SPILL);
        hipLaunchKernelGGL((k_numeric<T, IP, OFF, UB>), dim3(p.list_grid), dim3(BLOCK), 0, h->stream,
                           r0, n, p.B.cols, Ap, Aj, Ax, Bp, Bj, Bx, off, cj, cx, alpha, p.row_cnt,
                           p.seg, nz0, p.seg_len, (const int32_t*)l1, (const int32_t*)cnt);
    } else {
        PhaseTimer pt(h, SPG_PHASE_NUMERIC);
        hipLaunchKernelGGL((k_numeric<T, IP, OFF, UB>), dim3((unsigned)grid_for(n, WPB)), dim3(BLOCK), 0,
                           h->stream, r0, n, p.B.cols, Ap, Aj, Ax, Bp, Bj, Bx, off, cj, cx, alpha,
                           p.row_cnt, p.seg, nz0, p.seg_len, (const int32_t*)nullptr,
                           (const int32_t*)nullptr);
    }
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

template <typename OUT>
spg_status_t run_scan(spg_handle_t h, spg_plan_s& p, void* out, int mirror_n = 0) {
    // the row-pointer scan uses the second status region of the control block
    // (mirror_n > 0: the control words also go to the pinned buffer, for wait_mirror)
    return launch_scan<OUT>(h, p.A.rows, (const int64_t*)p.row_cnt, (OUT*)out,
                            p.scan_status + scan_tiles(p.A.rows) + 1, p.scalars, false, nullptr, nullptr,
                            mirror_n ? h->pinned : nullptr, mirror_n ? ++h->mirror_gen : 0, mirror_n);
}

// ------------------------------------------------------------------------ tile path
// Once per plan: the row-major boundary index (a temporary in the bitmap region) -> the
// tile-major segment table + symbolic-tile starts.
template <typename IP>
spg_status_t tile_build_index(spg_handle_t h, spg_plan_s& p) {
    if (p.tidx_built) return SPG_STATUS_SUCCESS;
    const IP* Bp = (const IP*)p.B.indptr;
    const int32_t* Bj = (const int32_t*)p.B.indices;
    const int R = 1 << (p.twss - p.tws);
    {
        const int Gp = (int)tiles_padded(p);
        timed_launch(h, SPG_PHASE_LAYOUT, k_tile_index<IP>, dim3((unsigned)grid_for(p.B.rows, 4)), dim3(256), p.B.rows,
                     Bp, Bj, p.tws, Gp, p.tidx);
        SPG_LAUNCHED(h);
        const int64_t n2 = p.B.rows * Gp + rec_groups(p);
        timed_launch(h, SPG_PHASE_LAYOUT, k_bt_count,
                     dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(n2, 256), 65536))), dim3(256),
                     p.B.rows, Gp, p.G, R, (const uint2*)p.tidx, p.tptr, p.sidx, p.rgs);
        SPG_LAUNCHED(h);
        timed_launch(h, SPG_PHASE_LAYOUT, k_bj16,
                     dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(p.B.nnz, 256), 65536))), dim3(256),
                     p.B.nnz, Bj, p.bj16);
        SPG_LAUNCHED(h);
    }
    spg_status_t st = launch_scan<int32_t, int32_t>(h, bt_entries(p), p.tptr, p.tptr, bt_scan_status(p),
                                                    p.scalars + 2, false);
    if (st) return st;
    p.tidx_built = true;
    return SPG_STATUS_SUCCESS;
}

// Symbolic tiles of chunk c -> its item counts and bitmaps, then the item offsets (a scan
// seeded with the previous chunk's total: offsets are C positions) and its rows' part of
// C's row pointer.  Totals alternate between two scalar slots; the last chunk's lands in
// scalars[0..1] (total, overflow), where spg_symbolic reads it.
template <typename IP>
spg_status_t tile_sym_chunk(spg_handle_t h, spg_plan_s& p, int64_t c) {
    const int64_t r0 = tile_chunk_r0(p, c), n = tile_chunk_r1(p, c) - r0;
    int64_t* items = tile_chunk_items(p, c);
    if (n > 0) {
        if (p.sym_seg)
            timed_launch(h, SPG_PHASE_SYMBOLIC, k_tile_sym_seg<IP>, dim3(tile_grid(n * sym_tiles(p), SEG_WPB)),
                         dim3(SEG_WPB * WAVE), r0, n, p.tws, p.G, p.twss, (const IP*)p.A.indptr,
                         (const int32_t*)p.A.indices, (const IP*)p.B.indptr, (const uint16_t*)p.bj16,
                         (const uint32_t*)p.sidx, tile_dense(p) ? (uint32_t*)nullptr : p.bitmap, items,
                         sym_full(p) ? p.B.cols : (int64_t)0);
        else if (SPG_SYM8 && SPG_SYM8_CW > 1)   // shared bitmap, SPG_SYM8_CW waves per task
            timed_launch(h, SPG_PHASE_SYMBOLIC, k_tile_sym8c<IP, SPG_SYM8_CW>,
                         dim3(coop_grid(n * sym_tiles(p), SPG_SYM8_CW)), dim3(SPG_SYM8_CW * WAVE),
                         r0, n, p.tws, p.G, p.twss, (const IP*)p.A.indptr, (const int32_t*)p.A.indices,
                         (const IP*)p.B.indptr, (const uint16_t*)p.bj16, (const uint32_t*)p.sidx,
                         tile_dense(p) ? (uint32_t*)nullptr : p.bitmap, items);
        else if (SPG_SYM8)
            timed_launch(h, SPG_PHASE_SYMBOLIC, k_tile_sym8<IP>, dim3(tile_grid(n * sym_tiles(p))), dim3(TILE_WPB * WAVE),
                         r0, n, p.tws, p.G, p.twss, (const IP*)p.A.indptr, (const int32_t*)p.A.indices,
                         (const IP*)p.B.indptr, (const uint16_t*)p.bj16, (const uint32_t*)p.sidx,
                         tile_dense(p) ? (uint32_t*)nullptr : p.bitmap, items);
        else
            timed_launch(h, SPG_PHASE_SYMBOLIC, k_tile_sym<IP>, dim3(tile_grid(n * sym_tiles(p))), dim3(TILE_WPB * WAVE),
                         r0, n, p.tws, p.G, p.twss, (const IP*)p.A.indptr, (const int32_t*)p.A.indices,
                         (const IP*)p.B.indptr, (const uint16_t*)p.bj16, (const uint32_t*)p.sidx,
                         tile_dense(p) ? (uint32_t*)nullptr : p.bitmap, items);
        SPG_LAUNCHED(h);
    }
    const int64_t nch = tile_chunks(p);
    int64_t* scal = c == nch - 1 ? p.scalars : p.scalars + 12 + 2 * (c & 1);
    const int64_t* seed = c == 0 ? nullptr : p.scalars + 12 + 2 * ((c - 1) & 1);
    return launch_scan<int64_t>(h, n * p.G, (const int64_t*)items, items, item_scan_status(p), scal,
                                true, nullptr, nullptr, nullptr, 0, 0, seed);
}

template <typename OUT>
spg_status_t tile_rowptr_chunk(spg_handle_t h, spg_plan_s& p, int64_t c, void* cp) {
    const int64_t r0 = tile_chunk_r0(p, c), n = tile_chunk_r1(p, c) - r0;
    timed_launch(h, SPG_PHASE_SCAN, k_items_to_rowptr<OUT>, dim3((unsigned)grid_for(n + 1, 256)), dim3(256), n, p.G,
                 (const int64_t*)tile_chunk_items(p, c), (OUT*)cp + r0);
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

// spg_symbolic on the tile path: every chunk's counts, offsets and row pointer.  A single
// chunk's offsets -- every chunk's on dense tiles -- stay valid for the numeric pass (and a
// repeated call only rewrites the row pointer); otherwise the numeric pass recomputes each
// chunk's.
template <typename IP, typename OUT>
spg_status_t tile_symbolic(spg_handle_t h, spg_plan_s& p, void* cp) {
    spg_status_t st;
    if ((st = tile_build_index<IP>(h, p))) return st;
    const int64_t nch = tile_chunks(p);
    if ((nch == 1 || tile_dense(p)) && p.counts_ready) {
        for (int64_t c = 0; c < nch; ++c)
            if ((st = tile_rowptr_chunk<OUT>(h, p, c, cp))) return st;
        return SPG_STATUS_SUCCESS;
    }
    for (int64_t c = 0; c < nch; ++c) {
        if ((st = tile_sym_chunk<IP>(h, p, c))) return st;
        if ((st = tile_rowptr_chunk<OUT>(h, p, c, cp))) return st;
    }
    return SPG_STATUS_SUCCESS;
}

// spg_numeric on the tile path: the tile-major B records once, then chunk by chunk (the
// chunk's counts, bitmaps and offsets again when there are several and the tiles are not
// dense) the numeric tiles.  spg_numeric_tiles (tm != nullptr, one chunk): the records'
// columns once, the values of column tiles [g0, g1) from the tile-major values `tm`, and
// only those tiles' items.
template <typename T, typename IP>
spg_status_t tile_numeric(spg_handle_t h, spg_plan_s& p, int32_t* cj, T* cx, T alpha, int64_t g0 = 0,
                          int64_t g1 = -1, const T* tm = nullptr) {
    if (g1 < 0) g1 = p.G;
    const IP* Ap = (const IP*)p.A.indptr;
    const IP* Bp = (const IP*)p.B.indptr;
    const int32_t* Aj = (const int32_t*)p.A.indices;
    const int32_t* Bj = (const int32_t*)p.B.indices;
    const T* Ax = (const T*)p.A.values;
    const T* Bx = (const T*)p.B.values;
    if (tm) {
        if (!p.brec_cols) {
            timed_launch(h, SPG_PHASE_LAYOUT, k_bt_pack<T, IP, 1>, dim3((unsigned)grid_for(p.B.rows, 4)), dim3(256),
                         p.B.rows, Bp, Bj, Bx, p.tws, (const int32_t*)p.tptr, (uint32_t*)p.brec, p.B.nnz, (T*)nullptr,
                         p.rgs);
            SPG_LAUNCHED(h);
            p.brec_cols = true;
        }
        p.brec_built = false;   // values of other tiles are stale for a later spg_numeric
        // records of groups [q0, q1) = [table word q0*W, word (q1-1)*W + W-1) -- the table is one
        // scan: group q's records start where group q-1's end (g0 and g1 are group-aligned)
        const int32_t* tp = (const int32_t*)p.tptr;
        const int64_t W = group_words(p);
        const int64_t q0 = g0 >> p.rgs, q1 = (g1 + (1 << p.rgs) - 1) >> p.rgs;
        const int64_t est = std::max<int64_t>(1, p.B.nnz * (q1 - q0) / std::max<int64_t>(rec_groups(p), 1));
        timed_launch(h, SPG_PHASE_LAYOUT, k_bt_fill<T>,
                     dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(est, 256), 16384))), dim3(256),
                     tp + q0 * W, tp + (q1 - 1) * W + (W - 1), tm, (uint32_t*)p.brec);
        SPG_LAUNCHED(h);
    } else if (!p.brec_built) {
        timed_launch(h, SPG_PHASE_LAYOUT, k_bt_pack<T, IP>, dim3((unsigned)grid_for(p.B.rows, 4)), dim3(256), p.B.rows,
                     Bp, Bj, Bx, p.tws, (const int32_t*)p.tptr, (uint32_t*)p.brec, p.B.nnz, (T*)nullptr, p.rgs);
        SPG_LAUNCHED(h);
        p.brec_built = true;
        p.brec_cols = true;
    }
    // byte offset of sentinel region r after B's records (k_bt_pack)
    auto sent = [&](int r) {
        return (uint32_t)(((uint64_t)p.B.nnz + (uint64_t)r * SENT_N) * (uint64_t)rec_bytes<T>());
    };
    const int64_t nch = tile_chunks(p);
    for (int64_t c = 0; c < nch; ++c) {
        spg_status_t st;
        if (nch > 1 && !tile_dense(p) && (st = tile_sym_chunk<IP>(h, p, c))) return st;
        const int64_t r0 = tile_chunk_r0(p, c), n = tile_chunk_r1(p, c) - r0;
        if (n <= 0) continue;
        // the items of tiles [g0, g1) (host keeps rows*G < 2^31); items of record groups
        // [g0 / RG, ceil(g1 / RG)) for the cooperative sparse kernel
        uint32_t it_lo = (uint32_t)(g0 * n), it_hi = (uint32_t)(g1 * n);
        int64_t nit = (g1 - g0) * n;
        KernelTimer kt(h, SPG_PHASE_NUMERIC);
        // dense accumulator when the tile fits one window; round groups (tile_variant())
        const bool dense = tile_dense(p);
        const int ru = tile_variant().ru;
        auto launch = [&](auto dn, auto rn) {
            constexpr bool DN = decltype(dn)::value;
            constexpr int RN = decltype(rn)::value;
            constexpr int WPBN = tile_num_wpb<DN>();
            hipExtLaunchKernelGGL((k_tile<T, IP, DN, RN>), dim3(tile_grid(nit, WPBN)), dim3(WPBN * WAVE), 0,
                                  h->stream, kt.a, kt.b, 0, r0, n, p.tws, p.G, Ap, Aj, Ax, p.B.rows,
                                  (const uint32_t*)p.brec, (const int32_t*)p.tptr,
                                  dense ? (const uint32_t*)nullptr : (const uint32_t*)p.bitmap,
                                  (const int64_t*)tile_chunk_items(p, c), cj, cx, alpha, it_lo, it_hi, p.rgs);
        };
        if constexpr (std::is_same<T, float>::value) {
            if (dense && fp32_runs(p)) {   // fp32 dense tiles of long B segments: entry runs
                hipExtLaunchKernelGGL((k_tile_dn<T, IP, 1024>), dim3(tile_grid(nit, DN_WPB)), dim3(DN_WPB * WAVE),
                                      0, h->stream, kt.a, kt.b, 0, r0, n, p.tws, p.G, Ap, Aj, Ax, p.B.rows,
                                      (const uint32_t*)p.brec, (const int32_t*)p.tptr,
                                      (const int64_t*)tile_chunk_items(p, c), cj, cx, alpha,
                                      sent(sentinel_region(1024)), it_lo, it_hi, p.rgs);
                SPG_LAUNCHED(h);
                continue;
            }
        }
        if constexpr (OrderedLdsAdd<T>::value) {
            if (!dense && p.lean && SPG_SP_LEAN) {   // sparse tiles, ordered LDS adds
                auto sp = [&](auto cfg, auto rgc) {
                    using CF = decltype(cfg);
                    constexpr int RG = decltype(rgc)::value;
                    if (RG > 1) {   // items (record group, row): one block of RG waves each
                        const int64_t q0 = g0 >> p.rgs, q1 = (g1 + RG - 1) >> p.rgs;
                        it_lo = (uint32_t)(q0 * n);
                        it_hi = (uint32_t)(q1 * n);
                        nit = (q1 - q0) * n;
                    }
                    // RG > 1: a persistent grid, 8 / RG blocks per CU (the LDS holds 8 such waves)
                    const unsigned spg_grid = RG > 1 ? (unsigned)std::min<int64_t>(coop_grid(nit, RG), (int64_t)h->cus * 8 / RG)
                                                     : coop_grid(nit, RG);
                    hipExtLaunchKernelGGL((k_tile_sp<T, IP, CF, RG>), dim3(spg_grid), dim3(RG * WAVE),
                                          0, h->stream, kt.a, kt.b, 0, r0, n, p.tws, p.G, Ap, Aj, Ax, p.B.rows,
                                          (const uint32_t*)p.brec, (const int32_t*)p.tptr, (const uint32_t*)p.bitmap,
                                          (const int64_t*)tile_chunk_items(p, c), cj, cx, alpha,
                                          sent(2), it_lo, it_hi, p.rgs);   // (sparse tiles' region)
                };
                using One = std::integral_constant<int, 1>;
                if constexpr (std::is_same<T, double>::value) {
                    bool done = false;
                    if constexpr (SPG_SP_RGS > 0) {
                        if (p.tws > 12 && p.rgs == SPG_SP_RGS) {
                            sp(SpCfgRG{}, std::integral_constant<int, (1 << SPG_SP_RGS)>{});
                            done = true;
                        }
                    }
                    if (!done) {
                        if (p.tws > 12) sp(SpCfg2048{}, One{});
                        else sp(SpCfg1024{}, One{});
                    }
                } else {
                    sp(SpCfg1024{}, One{});
                }
                SPG_LAUNCHED(h);
                continue;
            }
            if (dense && p.lean) {   // ordered LDS adds (spgemm_tile_dn.hpp)
                auto dn = [&](auto twd) {
                    constexpr int TWD = decltype(twd)::value;
                    if constexpr (SPG_DN_RGS > 0 && TWD == 2048) {
                        if (p.rgs == SPG_DN_RGS) {   // record groups of DN_WPB tiles, one per block
                            const int64_t q0 = g0 >> p.rgs, q1 = (g1 + DN_WPB - 1) >> p.rgs;
                            const unsigned gd = (unsigned)std::min<int64_t>(coop_grid((q1 - q0) * n, DN_WPB),
                                                                            SPG_DN_RG_PERSIST ? (int64_t)h->cus * 4 : ((int64_t)1 << 30));
                            hipExtLaunchKernelGGL((k_tile_dn<T, IP, TWD, DN_WPB>), dim3(gd), dim3(DN_WPB * WAVE),
                                                  0, h->stream, kt.a, kt.b, 0, r0, n, p.tws, p.G, Ap, Aj, Ax, p.B.rows,
                                                  (const uint32_t*)p.brec, (const int32_t*)p.tptr,
                                                  (const int64_t*)tile_chunk_items(p, c), cj, cx, alpha,
                                                  sent(sentinel_region(TWD)), (uint32_t)(q0 * n), (uint32_t)(q1 * n), p.rgs);
                            return;
                        }
                    }
                    hipExtLaunchKernelGGL((k_tile_dn<T, IP, TWD>), dim3(tile_grid(nit, DN_WPB)), dim3(DN_WPB * WAVE),
                                          0, h->stream, kt.a, kt.b, 0, r0, n, p.tws, p.G, Ap, Aj, Ax, p.B.rows,
                                          (const uint32_t*)p.brec, (const int32_t*)p.tptr,
                                          (const int64_t*)tile_chunk_items(p, c), cj, cx, alpha,
                                          sent(sentinel_region(TWD)), it_lo, it_hi, p.rgs);
                };
                if constexpr (std::is_same<T, double>::value) {
                    if constexpr (DN_TW_MAX > 2048) {
                        if ((1 << p.tws) > 2048) {
                            dn(std::integral_constant<int, DN_TW_MAX>{});
                            SPG_LAUNCHED(h);
                            continue;
                        }
                    }
                    if ((1 << p.tws) > 1024) dn(std::integral_constant<int, 2048>{});
                    else dn(std::integral_constant<int, 1024>{});
                } else {
                    dn(std::integral_constant<int, 1024>{});
                }
                SPG_LAUNCHED(h);
                continue;
            }
        }
        constexpr int UF = sizeof(T) > 8 ? 4 : 8;
        using D1 = std::integral_constant<bool, true>;
        using D0 = std::integral_constant<bool, false>;
        using R1 = std::integral_constant<int, 1>;
        using R2 = std::integral_constant<int, 2>;
        using RF = std::integral_constant<int, UF>;
        if (dense) {
            if (ru == 2) launch(D1{}, R2{}); else if (ru >= UF) launch(D1{}, RF{}); else launch(D1{}, R1{});
        } else {
            if (ru == 2) launch(D0{}, R2{}); else if (ru >= UF) launch(D0{}, RF{}); else launch(D0{}, R1{});
        }
        SPG_LAUNCHED(h);
    }
    return SPG_STATUS_SUCCESS;
}

// ALG1 single pass: structure + values + row pointer in one launch, compact into tj/tx
template <typename T, typename IP, typename OUT>
spg_status_t alg1_fused_run(spg_handle_t h, spg_plan_s& p, void* cp) {
    if (p.use_row) {
        // count pass (every row), row-pointer scan, one numeric pass into C's compact
        // arrays (estimate-sized: a total past `cap` writes nothing and is redone)
        // no memset of the control block: the count pass zeroes the scan's status words,
        // spills are counted in the handle's counter, which the scan moves into
        // scalars[5] and re-arms
        const unsigned grid = (unsigned)grid_for(p.A.rows, RowSmall::WPB * row_pair<ROW_LB>());
        const unsigned grid_sym = (unsigned)grid_for(p.A.rows, RowSmall::WPB * row_pair<ROW_SYM>());
        // the numeric launch's scan words: ticket + tile status, then the group prefixes
        unsigned long long* status = p.scan_status + scan_tiles(p.A.rows) + 1;
        const int64_t nscan = scan_tiles(p.A.rows);
        const int64_t nstatus = nscan + 1 + row_groups(p.A.rows);
        RowExt<IP>* ext = (RowExt<IP>*)p.ext;
        RowScan<OUT> sa{nscan, (OUT*)cp, status, status + nscan + 1, p.scalars, nullptr, nullptr, nullptr, 0, 0,
                        h->lb_spin};
        if (!p.counts_ready) {
            if (h->spill_ctr_dirty) SPG_HIP(h, hipMemsetAsync(h->spill_ctr, 0, sizeof(int32_t), h->stream));
            h->spill_ctr_dirty = true;
            timed_launch(h, SPG_PHASE_SYMBOLIC, k_row<double, IP, int64_t, ROW_SYM, RowSmall>, dim3(grid_sym), dim3(RowSmall::WPB * WAVE),
                               (int64_t)0, p.A.rows, p.B.cols, (const IP*)p.A.indptr,
                               (const int32_t*)p.A.indices, (const double*)nullptr, (const IP*)p.B.indptr,
                               (const int32_t*)p.B.indices, (const double*)nullptr, (const int64_t*)nullptr,
                               (int32_t*)nullptr, (double*)nullptr, 1.0, p.row_cnt, p.spill, h->spill_ctr,
                               (int)ROW_COUNT_ALL, (int64_t)0, (const int64_t*)nullptr, status, nstatus,
                               ext, RowScan<int64_t>{});
            SPG_LAUNCHED(h);
            // the scan blocks hand the spill count over (to scalars[5]), re-arm the counter and
            // mirror total / overflow / spills into the pinned buffer
            sa.move_cnt = h->spill_ctr;
            sa.move_dst = p.scalars + 5;
            sa.host_mirror = h->pinned;
            sa.mirror_gen = ++h->mirror_gen;
            sa.mirror_n = 2;   // words 0, 1 (+ 5: the move)
            h->spill_ctr_dirty = false;
        } else {   // repeated call: the first call already moved the spill count
            SPG_HIP(h, hipMemsetAsync(status, 0, sizeof(unsigned long long) * (size_t)nstatus, h->stream));
        }
        KernelTimer kt(h, SPG_PHASE_NUMERIC);
        hipExtLaunchKernelGGL((k_row<T, IP, OUT, ROW_LB, RowSmall>), dim3((unsigned)(nscan + grid)),
                              dim3(RowSmall::WPB * WAVE), 0, h->stream, kt.a, kt.b, 0, (int64_t)0, p.A.rows, p.B.cols,
                              (const IP*)p.A.indptr, (const int32_t*)p.A.indices, (const T*)p.A.values,
                              (const IP*)p.B.indptr, (const int32_t*)p.B.indices, (const T*)p.B.values,
                              (const OUT*)nullptr, p.tj, (T*)p.tx, (T)1, p.row_cnt, p.spill, spill_counts(p, true),
                              (int)ROW_LISTED, std::max<int64_t>(p.cap, 1), (const int64_t*)nullptr,
                              (unsigned long long*)nullptr, (int64_t)0, ext, sa);
        SPG_LAUNCHED(h);
        return SPG_STATUS_SUCCESS;
    }
    PhaseTimer pt(h, SPG_PHASE_NUMERIC);
    hipLaunchKernelGGL((k_short<T, IP, OUT, SHORT_NUMLB, ShortSmall>), dim3((unsigned)grid_for(p.A.rows, ShortSmall::WPB)),
                       dim3(ShortSmall::WPB * WAVE), 0, h->stream, (int64_t)0, p.A.rows, p.B.cols,
                       (const IP*)p.A.indptr, (const int32_t*)p.A.indices, (const T*)p.A.values,
                       (const IP*)p.B.indptr, (const int32_t*)p.B.indices, (const T*)p.B.values,
                       (const OUT*)nullptr, p.tj, (T*)p.tx, (T)1, p.row_cnt, (int32_t*)nullptr,
                       (int32_t*)nullptr, (const int32_t*)nullptr, (const int32_t*)nullptr, p.lb, (OUT*)cp,
                       p.scalars, p.cap);
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

// ALG1 single pass on k_row: values of the rows it spilled (at the row pointer it wrote)
template <typename T, typename IP, typename OUT>
spg_status_t alg1_fused_spills(spg_handle_t h, spg_plan_s& p, const void* cp) {
    PhaseTimer ps(h, SPG_PHASE_SPILL);
    hipLaunchKernelGGL((k_numeric<T, IP, OUT, false>), dim3(p.list_grid), dim3(BLOCK), 0, h->stream,
                       (int64_t)0, p.A.rows, p.B.cols, (const IP*)p.A.indptr, (const int32_t*)p.A.indices,
                       (const T*)p.A.values, (const IP*)p.B.indptr, (const int32_t*)p.B.indices,
                       (const T*)p.B.values, (const OUT*)cp, p.tj, (T*)p.tx, (T)1, p.row_cnt, p.seg,
                       (int64_t)0, p.seg_len, (const int32_t*)p.spill, (const int32_t*)(p.scalars + 5));
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

template <typename T, typename IP>
spg_status_t alg1_fused_typed(spg_handle_t h, spg_plan_s& p, void* cp, spg_index_t ct) {
    return ct == SPG_INDEX_64I ? alg1_fused_run<T, IP, int64_t>(h, p, cp) : alg1_fused_run<T, IP, int32_t>(h, p, cp);
}

template <typename IP>
spg_status_t symbolic_typed(spg_handle_t h, spg_plan_s& p) {
    spg_status_t st;
    if (p.alg == SPG_ALG3) {
        for (size_t c = 0; c + 1 < p.chunk_rows.size(); ++c) {
            if (c > 0 && p.use_short && p.nspc == 0)
                SPG_HIP(h, hipMemsetAsync(spill_counts(p, false), 0, 2 * sizeof(int32_t), h->stream));
            if ((st = run_symbolic_rows<IP>(h, p, p.chunk_rows[c], p.chunk_rows[c + 1], p.chunk_nz[c], (int)c)))
                return st;
        }
        return SPG_STATUS_SUCCESS;
    }
    return run_symbolic_rows<IP>(h, p, 0, p.A.rows, 0);
}

template <typename T, typename IP>
spg_status_t alg1_compute(spg_handle_t h, spg_plan_s& p) {
    // the fused structure+value pass at upper-bound offsets (the product prefix in p.ub,
    // computed when the plan was built)
    return run_numeric_rows<T, IP, int64_t, true>(h, p, 0, p.A.rows, 0, p.ub, p.tj, (T*)p.tx, (T)1);
}

template <typename T, typename IP, typename IPC>
spg_status_t numeric_typed(spg_handle_t h, spg_plan_s& p, const spg_csr_t& C, T alpha) {
    const IPC* cp = (const IPC*)C.indptr;
    if (p.alg1_fused) {
        // C already computed compact in tj/tx: copy (unless C points there) and scale
        const bool same = C.indices == (void*)p.tj && C.values == p.tx;
        if (same && alpha != (T)1) {
            if (p.scaled_in_place) return SPG_STATUS_INVALID_VALUE;   // would scale twice
            p.scaled_in_place = true;
        }
        if (!same || alpha != (T)1) {
            PhaseTimer pt(h, SPG_PHASE_COMPACT);
            hipLaunchKernelGGL(k_copy_scale<T>, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(p.nnzC, BLOCK), 65536))),
                               dim3(BLOCK), 0, h->stream, p.nnzC, (const int32_t*)p.tj, (const T*)p.tx,
                               (int32_t*)C.indices, (T*)C.values, alpha);
            SPG_LAUNCHED(h);
        }
        return SPG_STATUS_SUCCESS;
    }
    if (p.alg == SPG_ALG1 && !p.use_tile && !fused_alg1(p)) {
        if (p.A.rows > 0) {
            PhaseTimer pt(h, SPG_PHASE_COMPACT);
            hipLaunchKernelGGL((k_compact<T, IPC>), dim3((unsigned)grid_for(p.A.rows, WPB)), dim3(BLOCK), 0,
                               h->stream, p.A.rows, (const int64_t*)p.ub, cp, (const int32_t*)p.tj,
                               (const T*)p.tx, (int32_t*)C.indices, (T*)C.values, alpha);
            SPG_LAUNCHED(h);
        }
        return SPG_STATUS_SUCCESS;
    }
    spg_status_t st;
    if (p.use_tile) return tile_numeric<T, IP>(h, p, (int32_t*)C.indices, (T*)C.values, alpha);
    if (p.alg == SPG_ALG3) {
        for (size_t c = 0; c + 1 < p.chunk_rows.size(); ++c) {
            if (c > 0 && p.use_short && p.nspc == 0)
                SPG_HIP(h, hipMemsetAsync(spill_counts(p, true), 0, 2 * sizeof(int32_t), h->stream));
            if ((st = run_numeric_rows<T, IP, IPC, false>(h, p, p.chunk_rows[c], p.chunk_rows[c + 1],
                                                          p.chunk_nz[c], cp, (int32_t*)C.indices,
                                                          (T*)C.values, alpha, (int)c)))
                return st;
        }
        return SPG_STATUS_SUCCESS;
    }
    return run_numeric_rows<T, IP, IPC, false>(h, p, 0, p.A.rows, 0, cp, (int32_t*)C.indices,
                                               (T*)C.values, alpha);
}

template <typename IP>
spg_status_t validate_typed(spg_handle_t h, const spg_csr_t& M, int* flags) {
    if (M.rows > 0) {
        PhaseTimer pt(h, SPG_PHASE_VALIDATE);
        hipLaunchKernelGGL(k_validate<IP>, dim3((unsigned)grid_for(M.rows, BLOCK)), dim3(BLOCK), 0,
                           h->stream, M.rows, M.cols, M.nnz, (const IP*)M.indptr,
                           (const int32_t*)M.indices, flags);
        SPG_LAUNCHED(h);
    }
    return SPG_STATUS_SUCCESS;
}

}  // namespace

// =============================================================================== C ABI
// ---- 16-bit columns for the structure broadcast (include/spgemm.h, spg_cols16_*)
// One wave per row.  Split: every column's low half, and where the row's columns reach each
// interior block start c * 65536 (the first entry whose high half is >= c; the row length
// when none is).  Each start is written by exactly one lane: the entry whose high half
// steps over it, or the tail loop for blocks past the row's last column.
template <typename IP>
__global__ __launch_bounds__(256) void k_cols16_split(int64_t rows, const IP* __restrict__ Mp,
                                                      const int32_t* __restrict__ Mj, int nb1,
                                                      uint32_t* __restrict__ starts, uint16_t* __restrict__ lo16) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int l = lane_id();
    const int64_t b = (int64_t)Mp[row];
    const uint32_t len = (uint32_t)((int64_t)Mp[row + 1] - b);
    uint32_t* __restrict__ st = starts + row * nb1;
    for (uint32_t i = l; i < len; i += WAVE) {
        const uint32_t c = (uint32_t)Mj[b + i];
        lo16[b + i] = (uint16_t)(c & 0xffffu);
        const int hi = min((int)(c >> 16), nb1);   // (clamped: a column past M's width writes nothing past the row's starts)
        const int hp = i ? min((int)((uint32_t)Mj[b + i - 1] >> 16), nb1) : 0;
        for (int q = hp + 1; q <= hi; ++q) st[q - 1] = i;
    }
    const int hl = len ? (int)((uint32_t)Mj[b + len - 1] >> 16) : 0;
    for (int q = hl + 1 + l; q <= nb1; q += WAVE) st[q - 1] = len;
}

// Join: column = (block << 16) | low half, the block = the number of interior starts <= the
// entry's offset in its row (the starts ascend; a binary search over the row's nb1 starts).
template <typename IP>
__global__ __launch_bounds__(256) void k_cols16_join(int64_t rows, const IP* __restrict__ Mp, int nb1,
                                                     const uint32_t* __restrict__ starts,
                                                     const uint16_t* __restrict__ lo16, int32_t* __restrict__ Mj) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int l = lane_id();
    const int64_t b = (int64_t)Mp[row];
    const uint32_t len = (uint32_t)((int64_t)Mp[row + 1] - b);
    const uint32_t* __restrict__ st = starts + row * nb1;
    for (uint32_t i = l; i < len; i += WAVE) {
        int lo = 0, hi = nb1;   // first q with st[q] > i
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (st[mid] <= i) lo = mid + 1; else hi = mid;
        }
        Mj[b + i] = (int32_t)(((uint32_t)lo << 16) | (uint32_t)lo16[b + i]);
    }
}

extern "C" {

int spg_version(void) { return SPG_VERSION_MAJOR * 10000 + SPG_VERSION_MINOR * 100 + SPG_VERSION_PATCH; }

#ifndef SPG_SOURCE_ID
#define SPG_SOURCE_ID "unknown"
#endif
#ifndef SPG_HIPFLAGS
#define SPG_HIPFLAGS ""
#endif
const char* spg_build_info(void) { return "source_id=" SPG_SOURCE_ID " hipflags=" SPG_HIPFLAGS; }

const char* spg_status_string(spg_status_t s) {
    switch (s) {
        case SPG_STATUS_SUCCESS: return "SPG_STATUS_SUCCESS";
        case SPG_STATUS_NOT_INITIALIZED: return "SPG_STATUS_NOT_INITIALIZED";
        case SPG_STATUS_ALLOC_FAILED: return "SPG_STATUS_ALLOC_FAILED";
        case SPG_STATUS_INVALID_VALUE: return "SPG_STATUS_INVALID_VALUE";
        case SPG_STATUS_ARCH_MISMATCH: return "SPG_STATUS_ARCH_MISMATCH";
        case SPG_STATUS_EXECUTION_FAILED: return "SPG_STATUS_EXECUTION_FAILED";
        case SPG_STATUS_INTERNAL_ERROR: return "SPG_STATUS_INTERNAL_ERROR";
        case SPG_STATUS_NOT_SUPPORTED: return "SPG_STATUS_NOT_SUPPORTED";
        case SPG_STATUS_INSUFFICIENT_RESOURCES: return "SPG_STATUS_INSUFFICIENT_RESOURCES";
        case SPG_STATUS_OVERFLOW: return "SPG_STATUS_OVERFLOW";
        case SPG_STATUS_HIP_ERROR: return "SPG_STATUS_HIP_ERROR";
    }
    return "SPG_STATUS_UNKNOWN";
}

spg_status_t spg_create(spg_handle_t* handle, int hip_device) {
    if (!handle) return SPG_STATUS_INVALID_VALUE;
    *handle = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SPG_STATUS_NOT_INITIALIZED;
    int dev = hip_device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) return SPG_STATUS_NOT_INITIALIZED;
    }
    if (dev >= ndev) return SPG_STATUS_INVALID_VALUE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return SPG_STATUS_NOT_INITIALIZED;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SPG_STATUS_ARCH_MISMATCH;
    spg_handle_s* h = new (std::nothrow) spg_handle_s();
    if (!h) return SPG_STATUS_ALLOC_FAILED;
    h->device = dev;
    h->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (const char* e = std::getenv("SPG_LB_SPIN_TICKS")) h->lb_spin = std::strtoull(e, nullptr, 10);
    DeviceGuard dg_(dev);   // the handle's allocations on its device; the caller's device stays current
    hipError_t e = dg_.err;
    if (e == hipSuccess) e = lds_order_check(&h->lds_ordered, &h->lds_ordered32);
    if (const char* o = std::getenv("SPG_LDS_ORDERED"))
        if (std::strcmp(o, "0") == 0) h->lds_ordered = h->lds_ordered32 = false;
    // fine-grained (coherent) host memory: the scan's system-scope stores of the scalars and
    // then the generation word become visible to the polling host in that order
    // (wait_mirror); the default host allocation is coarse-grained unless HIP_HOST_COHERENT=1
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&h->pinned, PINNED_WORDS * sizeof(int64_t), hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) std::memset(h->pinned, 0, PINNED_WORDS * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc((void**)&h->spill_ctr, 256);
    if (e == hipSuccess) e = hipMemset(h->spill_ctr, 0, 256);
    if (e != hipSuccess) {
        delete h;
        return e == hipErrorOutOfMemory ? SPG_STATUS_ALLOC_FAILED : SPG_STATUS_HIP_ERROR;
    }
    *handle = h;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_destroy(spg_handle_t h) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    (void)hipStreamSynchronize(h->stream);   // an ALG1 call returns with its numeric pass queued
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->pinned) (void)hipHostFree(h->pinned);
    if (h->spill_ctr) (void)hipFree(h->spill_ctr);
    for (auto& q : h->pending) { (void)hipEventDestroy(q.a); (void)hipEventDestroy(q.b); }
    for (hipEvent_t e : h->pool) (void)hipEventDestroy(e);
    delete h;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_set_stream(spg_handle_t h, void* stream) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    // work still queued on the old stream may use the handle's scratch: drain it first
    if ((hipStream_t)stream != h->stream) SPG_HIP(h, hipStreamSynchronize(h->stream));
    h->stream = (hipStream_t)stream;
    return SPG_STATUS_SUCCESS;
}

int spg_last_hip_error(spg_handle_t h) { return h ? h->last_hip : 0; }

spg_status_t spg_plan(spg_handle_t h, const spg_csr_t* A, const spg_csr_t* B, spg_alg_t alg,
                      float chunk_fraction, size_t* workspace_bytes, void* workspace,
                      spg_plan_t* plan) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!workspace_bytes) return SPG_STATUS_INVALID_VALUE;
    spg_status_t st;
    if ((st = check_csr(A)) || (st = check_csr(B))) return st;
    if (A->cols != B->rows) return SPG_STATUS_INVALID_VALUE;
    if (A->value_type != B->value_type) return SPG_STATUS_INVALID_VALUE;
    if (A->indptr_type != B->indptr_type) return SPG_STATUS_INVALID_VALUE;
    if (alg != SPG_ALG_DEFAULT && alg != SPG_ALG1 && alg != SPG_ALG2 && alg != SPG_ALG3)
        return SPG_STATUS_INVALID_VALUE;
    if (alg == SPG_ALG3 && !(chunk_fraction > 0.0f && chunk_fraction <= 1.0f))
        return SPG_STATUS_INVALID_VALUE;
    if (workspace && !plan) return SPG_STATUS_INVALID_VALUE;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);

    spg_plan_s tmp;
    tmp.A = *A;
    tmp.B = *B;
    tmp.alg = alg == SPG_ALG_DEFAULT ? SPG_ALG2 : alg;
    tmp.cf = chunk_fraction;
    tmp.seg_len = A->nnz;
    tmp.use_short = want_short(*A, *B);
    tmp.use_row = row_kernel_enabled();
    tmp.lean = SPG_TILE_LEAN && h->lds_ordered;
    tmp.lean32 = SPG_TILE_LEAN && h->lds_ordered32;
    tmp.use_tile = !tmp.use_short && want_tile(*A, *B, tmp.tws, tmp.G, tmp.lean);
    if (tmp.use_tile) {
        tmp.TR = 1;
        tmp.twss = sym_tile_log2(*B, tmp.tws, &tmp.sym_seg);
        tmp.rgs = record_group_log2(tmp);
    }
    // the general kernel's launch over the spill list (rows the short kernels hand over: A
    // rows > 64 entries, C wider than 16384 columns, or a row whose repeated columns overflow
    // the register path's list -- narrow C rows, e.g. N = 1024 at density 0.01, where dozens of
    // rows spill).  It runs only when the list is non-empty; one wave per 16 rows of A up to
    // 1024 waves, so the listed rows run side by side (one 4-wave block per 1024 rows put
    // them in series: 96 us for the N = 1024 fp32 product above, against 37 us without spills)
    tmp.list_grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(256, grid_for(A->rows, 64)));
    // ALG1 and ALG3 size their buffers / chunks from the product counts, which needs the
    // device once.  The size query and the building call of one plan see the same
    // operands, so the building call reuses what the query measured.
    const bool same_as_query = h->q_valid && h->q_alg == tmp.alg && h->q_cf == chunk_fraction &&
                               std::memcmp(&h->q_A, A, sizeof(spg_csr_t)) == 0 &&
                               std::memcmp(&h->q_B, B, sizeof(spg_csr_t)) == 0;
    if (fused_alg1(tmp)) {
        // single pass: the output buffer is sized from the expected product count (no device
        // pass, no sync); a product that outgrows it is redone two-phase by spg_symbolic
        const double avgB = B->rows > 0 ? (double)B->nnz / (double)B->rows : 0.0;
        const double est = 1.15 * (double)A->nnz * avgB + 4096.0;
        const double full = (double)A->rows * (double)B->cols;
        tmp.cap = (int64_t)std::min(est, full);
    } else if (tmp.alg == SPG_ALG1 && !tmp.use_tile) {
        if (workspace && same_as_query) {
            tmp.P = h->q_P;
        } else if ((st = products_total(h, *A, *B, &tmp.P))) {
            return st;
        }
    } else if (tmp.alg == SPG_ALG3) {
        if (workspace && same_as_query) {
            tmp.P = h->q_P;
            tmp.chunk_rows = h->q_chunk_rows;
            tmp.chunk_nz = h->q_chunk_nz;
            tmp.seg_len = h->q_seg_len;
        } else {
            // The ALG3 cap: chunk_fraction of the single-pass (ALG1) buffer, P entries of
            // C's (index, value) pairs -- the working set cuSPARSE's ALG3 trades time against
            // (estimateMemory, spgemm_from_txt_alg3.cu:195-202).  When the unchunked
            // workspace is already within it, chunking would only add launches: one chunk,
            // decided from P alone (one scalar read back), without the per-row product
            // prefix and the row pointer the chunk cut needs on the host.
            spg_plan_s whole = tmp;
            whole.chunk_rows.assign({0, A->rows});
            whole.chunk_nz.assign({0, A->nnz});
            whole.seg_len = tmp.use_tile ? 1 : A->nnz;
            // (SPG_ALG3_CHUNK_ALWAYS=1 keeps the chunks regardless: a schedule-only switch the
            // GPU tests use to cover the chunked paths on small inputs; results are identical)
            const char* ae = std::getenv("SPG_ALG3_CHUNK_ALWAYS");
            const bool always = ae && std::strcmp(ae, "1") == 0;
            if ((st = products_total(h, *A, *B, &tmp.P))) return st;
            const double cap = (double)chunk_fraction * (double)std::max<int64_t>(tmp.P, 0) *
                               (double)(sizeof(int32_t) + vbytes(A->value_type));
            if (always || (double)make_layout(whole).total > cap) {
                if ((st = plan_chunks(h, tmp))) return st;
            } else {
                tmp.chunk_rows = whole.chunk_rows;
                tmp.chunk_nz = whole.chunk_nz;
                tmp.seg_len = whole.seg_len;
            }
        }
    }
    if (tmp.use_tile) tmp.seg_len = 1;   // no cursor scratch on the tile path
    if (tmp.use_short && tmp.use_row && (tmp.alg == SPG_ALG2 || tmp.alg == SPG_ALG3)) {
        const int64_t nch = tmp.alg == SPG_ALG3 ? (int64_t)tmp.chunk_rows.size() - 1 : 1;
        if (nch >= 1 && nch <= MIRROR_GEN_WORD - 16) tmp.nspc = nch;   // words 16.. stay below the generation word
    }
    if (!workspace) {
        h->q_valid = true;
        h->q_A = *A;
        h->q_B = *B;
        h->q_alg = tmp.alg;
        h->q_cf = chunk_fraction;
        h->q_P = tmp.P;
        h->q_chunk_rows = tmp.chunk_rows;
        h->q_chunk_nz = tmp.chunk_nz;
        h->q_seg_len = tmp.seg_len;
    }
    const Layout L = make_layout(tmp);
    if (!workspace) {
        *workspace_bytes = L.total;
        return SPG_STATUS_SUCCESS;
    }
    if (*workspace_bytes < L.total) return SPG_STATUS_INVALID_VALUE;
    spg_plan_s* p = new (std::nothrow) spg_plan_s(std::move(tmp));
    if (!p) return SPG_STATUS_ALLOC_FAILED;
    p->ws = (char*)workspace;
    p->ws_bytes = *workspace_bytes;
    carve(*p, L);
    // control block: scalars + spill counters + scan status words, zeroed once per plan
    {
        // (ALG1 on k_row zeroes what it uses itself)
        hipError_t e1 = fused_alg1(*p) && p->use_row ? hipSuccess
                                                     : hipMemsetAsync(p->ws, 0, L.row_cnt, h->stream);
        if (e1 != hipSuccess) { delete p; return hip_fail(h, e1); }
    }
    if (p->alg == SPG_ALG1 && !p->use_tile && !fused_alg1(*p)) {
        // upper-bound offsets for the single pass: product prefix straight into the workspace
        spg_status_t st2 = products_prefix(h, p->A, p->B, p->row_cnt, p->ub, p->scalars + 2,
                                           p->scan_status, false);
        if (st2) { delete p; return st2; }
    }
    *plan = p;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_num_products(spg_handle_t h, spg_plan_t p, int64_t* num_products) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p || !num_products) return SPG_STATUS_INVALID_VALUE;
    if (p->P < 0) {
        DeviceGuard dg_(h->device);
        SPG_HIP(h, dg_.err);
        spg_status_t st;
        if ((st = products_total(h, p->A, p->B, &p->P))) return st;
    }
    *num_products = p->P;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_symbolic(spg_handle_t h, spg_plan_t p, void* C_indptr, spg_index_t C_indptr_type,
                          int64_t* nnzC) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p || !C_indptr || !nnzC) return SPG_STATUS_INVALID_VALUE;
    if (C_indptr_type != SPG_INDEX_32I && C_indptr_type != SPG_INDEX_64I) return SPG_STATUS_INVALID_VALUE;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    spg_status_t st;
    const bool i64 = p->A.indptr_type == SPG_INDEX_64I;
    if (fused_alg1(*p) && !p->fused_failed && p->use_row) {
        // ALG1 on k_row: count pass (first call only), row-pointer scan, numeric pass into
        // the workspace's compact C -- no host sync in between.  A repeated call (the int64
        // retry after an int32 overflow, when the numeric pass wrote nothing) redoes the
        // scan and the numeric pass.
        st = dispatch_value(p->A.value_type, [&](auto tag) {
            using T = decltype(tag);
            return i64 ? alg1_fused_typed<T, int64_t>(h, *p, C_indptr, C_indptr_type)
                       : alg1_fused_typed<T, int32_t>(h, *p, C_indptr, C_indptr_type);
        });
        if (st) return st;
        int64_t sc[6];
        if (!p->counts_ready) {
            // the scan mirrored total / overflow / spills into the pinned buffer: wait for
            // that (no device->host copy, no wait for the numeric pass)
            if ((st = wait_mirror(h))) return st;
            for (int i = 0; i < 6; ++i) sc[i] = ((volatile int64_t*)h->pinned)[i];
        } else if ((st = read_scalars(h, p->scalars, 6, sc))) {
            return st;
        }
        p->counts_ready = true;
        if (sc[1]) return SPG_STATUS_OVERFLOW;   // int32 row pointer: retry with int64
        if (sc[0] <= p->cap) {
            p->alg1_fused = true;
            if ((int32_t)(sc[5] & 0xffffffffu) > 0) {   // the listed rows' values, at Cp
                st = dispatch_value(p->A.value_type, [&](auto tag) {
                    using T = decltype(tag);
                    if (i64)
                        return C_indptr_type == SPG_INDEX_64I ? alg1_fused_spills<T, int64_t, int64_t>(h, *p, C_indptr)
                                                              : alg1_fused_spills<T, int64_t, int32_t>(h, *p, C_indptr);
                    return C_indptr_type == SPG_INDEX_64I ? alg1_fused_spills<T, int32_t, int64_t>(h, *p, C_indptr)
                                                          : alg1_fused_spills<T, int32_t, int32_t>(h, *p, C_indptr);
                });
                if (st) return st;
            }
            p->nnzC = sc[0];
            p->c_indptr = C_indptr;
            p->c_indptr_type = C_indptr_type;
            *nnzC = sc[0];
            return SPG_STATUS_SUCCESS;
        }
        // an output larger than the estimate: redo the numeric pass into C (the counts and
        // the row pointer are valid)
        p->fused_failed = true;
        p->symbolic_runs = 1;
        p->sym_spills = (int64_t)(uint32_t)(sc[5] & 0xffffffffu);   // the numeric pass relists them
        SPG_HIP(h, hipMemsetAsync(p->scalars + 4, 0, 2 * sizeof(int64_t), h->stream));
        p->nnzC = sc[0];
        p->c_indptr = C_indptr;
        p->c_indptr_type = C_indptr_type;
        *nnzC = sc[0];
        return SPG_STATUS_SUCCESS;
    }
    if (fused_alg1(*p) && !p->fused_failed) {
        // ALG1 single pass: one launch writes C compact into tj/tx and its row pointer; a
        // repeated call (int64 retry) only rescans the row counts it recorded
        ++p->symbolic_runs;
        if (!p->counts_ready) {
            st = dispatch_value(p->A.value_type, [&](auto tag) {
                using T = decltype(tag);
                return i64 ? alg1_fused_typed<T, int64_t>(h, *p, C_indptr, C_indptr_type)
                           : alg1_fused_typed<T, int32_t>(h, *p, C_indptr, C_indptr_type);
            });
        } else {
            const int64_t tiles = scan_tiles(p->A.rows) + 1;
            SPG_HIP(h, hipMemsetAsync(p->scan_status + tiles, 0, sizeof(unsigned long long) * tiles, h->stream));
            st = C_indptr_type == SPG_INDEX_64I ? run_scan<int64_t>(h, *p, C_indptr)
                                                : run_scan<int32_t>(h, *p, C_indptr);
            if (!st) {   // the scan leaves the total in scalars[0]
                int64_t tot;
                if ((st = read_scalars(h, p->scalars, 1, &tot))) return st;
                if (C_indptr_type == SPG_INDEX_32I && tot > 2147483647LL) return SPG_STATUS_OVERFLOW;
                p->nnzC = tot;
                p->c_indptr = C_indptr;
                p->c_indptr_type = C_indptr_type;
                *nnzC = tot;
                return SPG_STATUS_SUCCESS;
            }
        }
        if (st) return st;
        int64_t sc[11];
        if ((st = read_scalars(h, p->scalars, 11, sc))) return st;
        if (!sc[LB_FAIL] && !sc[LB_CAPX]) {
            p->counts_ready = true;
            p->alg1_fused = true;
            const int64_t tot = sc[LB_TOTAL];
            if (C_indptr_type == SPG_INDEX_32I && tot > 2147483647LL) return SPG_STATUS_OVERFLOW;
            // k_row spilled rows (counted, row pointer written): their values, at that offset
            if (p->use_row && (int32_t)(sc[5] & 0xffffffffu) > 0) {
                st = dispatch_value(p->A.value_type, [&](auto tag) {
                    using T = decltype(tag);
                    if (i64)
                        return C_indptr_type == SPG_INDEX_64I ? alg1_fused_spills<T, int64_t, int64_t>(h, *p, C_indptr)
                                                              : alg1_fused_spills<T, int64_t, int32_t>(h, *p, C_indptr);
                    return C_indptr_type == SPG_INDEX_64I ? alg1_fused_spills<T, int32_t, int64_t>(h, *p, C_indptr)
                                                          : alg1_fused_spills<T, int32_t, int32_t>(h, *p, C_indptr);
                });
                if (st) return st;
            }
            p->nnzC = tot;
            p->c_indptr = C_indptr;
            p->c_indptr_type = C_indptr_type;
            *nnzC = tot;
            return SPG_STATUS_SUCCESS;
        }
        // a row the single pass cannot take, or an output larger than the estimate: redo
        // the product two-phase (symbolic + scan here, numeric straight into C)
        p->fused_failed = true;
        p->symbolic_runs = 0;
    }
    if (p->use_tile) {
        // counts, offsets and row pointer chunk by chunk; the last scan leaves the total in
        // scalars[0] (overflow of an int32 row pointer is checked here)
        st = i64 ? (C_indptr_type == SPG_INDEX_64I ? tile_symbolic<int64_t, int64_t>(h, *p, C_indptr)
                                                   : tile_symbolic<int64_t, int32_t>(h, *p, C_indptr))
                 : (C_indptr_type == SPG_INDEX_64I ? tile_symbolic<int32_t, int64_t>(h, *p, C_indptr)
                                                   : tile_symbolic<int32_t, int32_t>(h, *p, C_indptr));
        if (st) return st;
        int64_t tot;
        if ((st = read_scalars(h, p->scalars, 1, &tot))) return st;
        p->counts_ready = true;
        if (C_indptr_type == SPG_INDEX_32I && tot > 2147483647LL) return SPG_STATUS_OVERFLOW;
        p->nnzC = tot;
        p->c_indptr = C_indptr;
        p->c_indptr_type = C_indptr_type;
        *nnzC = tot;
        return SPG_STATUS_SUCCESS;
    }
    if (p->symbolic_runs++ > 0 && !p->use_tile) {
        // a repeated call (e.g. retrying with int64 row pointers): the row counts are kept;
        // re-arm the row-pointer scan's status words
        const int64_t tiles = scan_tiles(p->A.rows) + 1;
        SPG_HIP(h, hipMemsetAsync(p->scan_status + tiles, 0, sizeof(unsigned long long) * tiles, h->stream));
    }
    if (!p->counts_ready) {
        if (p->alg == SPG_ALG1 && !p->use_tile && !fused_alg1(*p)) {
            st = dispatch_value(p->A.value_type, [&](auto tag) {
                using T = decltype(tag);
                return i64 ? alg1_compute<T, int64_t>(h, *p) : alg1_compute<T, int32_t>(h, *p);
            });
        } else {
            st = i64 ? symbolic_typed<int64_t>(h, *p) : symbolic_typed<int32_t>(h, *p);
        }
        if (st) return st;
    }
    // the row-pointer scan mirrors the control words (+ every chunk's spill count) into the
    // pinned buffer: no device->host copy
    const bool chunks = p->nspc > 0 && !p->counts_ready;
    const int nread = chunks ? 16 + p->nspc : 5;
    st = C_indptr_type == SPG_INDEX_64I ? run_scan<int64_t>(h, *p, C_indptr, nread)
                                        : run_scan<int32_t>(h, *p, C_indptr, nread);
    if (st) return st;
    std::vector<int64_t> all((size_t)nread);
    if ((st = wait_mirror(h))) return st;
    for (int i = 0; i < nread; ++i) all[(size_t)i] = ((volatile int64_t*)h->pinned)[i];
    int64_t sc[5];
    for (int i = 0; i < 5; ++i) sc[i] = all[(size_t)i];
    if (chunks) {
        p->chunk_spills.assign(all.begin() + 16, all.end());
        for (auto& v : p->chunk_spills) v &= 0xffffffffLL;
    }
    // the short-row kernel spills the same rows in both passes: none in the symbolic pass
    // (one launch over all rows) means the numeric spill launch can be skipped
    if (p->use_short && (p->alg == SPG_ALG2 || fused_alg1(*p))) p->sym_spills = (int64_t)(uint32_t)(sc[4] & 0xffffffffu);
    p->counts_ready = true;      // counts stay valid for a repeated call
    if (sc[1]) return SPG_STATUS_OVERFLOW;
    p->nnzC = sc[0];
    p->c_indptr = C_indptr;
    p->c_indptr_type = C_indptr_type;
    *nnzC = sc[0];
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_numeric(spg_handle_t h, spg_plan_t p, const void* alpha, spg_csr_t* C) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p || !alpha || !C) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC < 0) return SPG_STATUS_NOT_INITIALIZED;     // spg_symbolic first
    if (C->rows != p->A.rows || C->cols != p->B.cols) return SPG_STATUS_INVALID_VALUE;
    if (C->value_type != p->A.value_type) return SPG_STATUS_INVALID_VALUE;
    if (C->indptr != p->c_indptr || C->indptr_type != p->c_indptr_type) return SPG_STATUS_INVALID_VALUE;
    if (C->nnz != p->nnzC) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC > 0 && (!C->indices || !C->values)) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC == 0) return SPG_STATUS_SUCCESS;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    const bool i64 = p->A.indptr_type == SPG_INDEX_64I;
    const bool c64 = C->indptr_type == SPG_INDEX_64I;
    return dispatch_value(p->A.value_type, [&](auto tag) {
        using T = decltype(tag);
        T a;
        std::memcpy(&a, alpha, sizeof(T));   // host value of C's type (a (re, im) pair if complex)
        if (i64) return c64 ? numeric_typed<T, int64_t, int64_t>(h, *p, *C, a)
                            : numeric_typed<T, int64_t, int32_t>(h, *p, *C, a);
        return c64 ? numeric_typed<T, int32_t, int64_t>(h, *p, *C, a)
                   : numeric_typed<T, int32_t, int32_t>(h, *p, *C, a);
    });
}

// ---- the numeric phase by column-tile groups (include/spgemm.h; multi-GPU B-value pipelining)
// The segment tables are built by spg_symbolic, or here on first use: a plan's values can
// be laid out tile-major (and their offsets read) before its symbolic pass, so the multi-GPU
// step sends them while the symbolic pass runs.  (Call under the handle's DeviceGuard.)
static spg_status_t tiles_supported(spg_handle_t h, spg_plan_t p) {
    if (!p) return SPG_STATUS_INVALID_VALUE;
    if (!p->use_tile || tile_chunks(*p) != 1 || p->alg1_fused) return SPG_STATUS_NOT_SUPPORTED;
    if (p->tidx_built) return SPG_STATUS_SUCCESS;
    return p->A.indptr_type == SPG_INDEX_64I ? tile_build_index<int64_t>(h, *p) : tile_build_index<int32_t>(h, *p);
}

spg_status_t spg_tile_value_offsets(spg_handle_t h, spg_plan_t p, int64_t* offsets, int64_t capacity) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p) return SPG_STATUS_INVALID_VALUE;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    spg_status_t st = tiles_supported(h, p);
    if (st) return st;
    const int64_t Gq = rec_groups(*p);   // value tiles = record groups
    if (capacity < Gq + 1 || !offsets) return SPG_STATUS_INVALID_VALUE;
    // group q starts at table word q*W; the last group's end slot holds nnz(B)
    const int64_t W = group_words(*p);
    std::vector<int32_t> w((size_t)Gq + 1);
    SPG_HIP(h, hipMemcpy2DAsync(w.data(), sizeof(int32_t), p->tptr, (size_t)W * sizeof(int32_t), sizeof(int32_t),
                                (size_t)Gq, hipMemcpyDeviceToHost, h->stream));
    SPG_HIP(h, hipMemcpyAsync(w.data() + Gq, (const int32_t*)p->tptr + (Gq - 1) * W + (W - 1),
                              sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
    SPG_HIP(h, hipStreamSynchronize(h->stream));
    for (int64_t g = 0; g <= Gq; ++g) offsets[g] = w[(size_t)g];
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_tile_values(spg_handle_t h, spg_plan_t p, void* tm) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p) return SPG_STATUS_INVALID_VALUE;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    spg_status_t st = tiles_supported(h, p);
    if (st) return st;
    if (!tm && p->B.nnz > 0) return SPG_STATUS_INVALID_VALUE;
    if (p->B.nnz > 0 && !p->B.values) return SPG_STATUS_INVALID_VALUE;
    if (p->B.rows == 0 || p->B.nnz == 0) return SPG_STATUS_SUCCESS;
    const bool i64 = p->A.indptr_type == SPG_INDEX_64I;
    return dispatch_value(p->A.value_type, [&](auto tag) {
        using T = decltype(tag);
        auto go = [&](auto ip) {
            using IP = decltype(ip);
            timed_launch(h, SPG_PHASE_LAYOUT, k_bt_pack<T, IP, 2>, dim3((unsigned)grid_for(p->B.rows, 4)), dim3(256),
                         p->B.rows, (const IP*)p->B.indptr, (const int32_t*)p->B.indices, (const T*)p->B.values,
                         p->tws, (const int32_t*)p->tptr, (uint32_t*)p->brec, p->B.nnz, (T*)tm, p->rgs);
        };
        if (i64) go(int64_t{}); else go(int32_t{});
        SPG_LAUNCHED(h);
        return SPG_STATUS_SUCCESS;
    });
}

spg_status_t spg_numeric_tiles(spg_handle_t h, spg_plan_t p, const void* alpha, spg_csr_t* C, const void* tm,
                               int64_t g0, int64_t g1) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!p || !alpha || !C) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC < 0) return SPG_STATUS_NOT_INITIALIZED;     // spg_symbolic first
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    spg_status_t st = tiles_supported(h, p);   // (spg_symbolic built the tables)
    if (st) return st;
    if (g0 < 0 || g1 > rec_groups(*p) || g0 > g1) return SPG_STATUS_INVALID_VALUE;   // value tiles
    if (C->rows != p->A.rows || C->cols != p->B.cols) return SPG_STATUS_INVALID_VALUE;
    if (C->value_type != p->A.value_type) return SPG_STATUS_INVALID_VALUE;
    if (C->indptr != p->c_indptr || C->indptr_type != p->c_indptr_type) return SPG_STATUS_INVALID_VALUE;
    if (C->nnz != p->nnzC) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC > 0 && (!C->indices || !C->values)) return SPG_STATUS_INVALID_VALUE;
    if (p->B.nnz > 0 && !tm) return SPG_STATUS_INVALID_VALUE;
    if (p->nnzC == 0 || g0 == g1) return SPG_STATUS_SUCCESS;
    const bool i64 = p->A.indptr_type == SPG_INDEX_64I;
    return dispatch_value(p->A.value_type, [&](auto tag) {
        using T = decltype(tag);
        T a;
        std::memcpy(&a, alpha, sizeof(T));
        // value tiles [g0, g1) = numeric tiles [g0 * RG, min(G, g1 * RG))
        const int64_t t0 = g0 << p->rgs, t1 = std::min<int64_t>(p->G, g1 << p->rgs);
        return i64 ? tile_numeric<T, int64_t>(h, *p, (int32_t*)C->indices, (T*)C->values, a, t0, t1, (const T*)tm)
                   : tile_numeric<T, int32_t>(h, *p, (int32_t*)C->indices, (T*)C->values, a, t0, t1, (const T*)tm);
    });
}

spg_status_t spg_spmv(spg_handle_t h, const spg_csr_t* A, const void* x, const void* alpha,
                      const void* beta, void* y) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    spg_status_t st = check_csr(A);
    if (st) return st;
    if (!alpha || !beta || (A->rows > 0 && !y) || (A->cols > 0 && A->nnz > 0 && !x))
        return SPG_STATUS_INVALID_VALUE;
    if (A->rows == 0) return SPG_STATUS_SUCCESS;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    const bool i64 = A->indptr_type == SPG_INDEX_64I;
    return dispatch_value(A->value_type, [&](auto tag) {
        using T = decltype(tag);
        T al, be;
        std::memcpy(&al, alpha, sizeof(T));
        std::memcpy(&be, beta, sizeof(T));
        const unsigned grid = (unsigned)grid_for(A->rows, SPMV_WPB * WAVE);
        PhaseTimer pt(h, SPG_PHASE_SPMV);
        if (i64)
            hipLaunchKernelGGL((k_spmv<T, int64_t>), dim3(grid), dim3(SPMV_WPB * WAVE), 0, h->stream, A->rows,
                               (const int64_t*)A->indptr, (const int32_t*)A->indices, (const T*)A->values,
                               (const T*)x, al, be, (T*)y);
        else
            hipLaunchKernelGGL((k_spmv<T, int32_t>), dim3(grid), dim3(SPMV_WPB * WAVE), 0, h->stream, A->rows,
                               (const int32_t*)A->indptr, (const int32_t*)A->indices, (const T*)A->values,
                               (const T*)x, al, be, (T*)y);
        SPG_LAUNCHED(h);
        return SPG_STATUS_SUCCESS;
    });
}

spg_status_t spg_result_in_workspace(spg_plan_t p, void** indices, void** values) {
    if (!p || !indices || !values) return SPG_STATUS_INVALID_VALUE;
    *indices = p->alg1_fused ? (void*)p->tj : nullptr;
    *values = p->alg1_fused ? p->tx : nullptr;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_peak_bytes(spg_plan_t p, size_t* bytes) {
    if (!p || !bytes) return SPG_STATUS_INVALID_VALUE;
    const size_t ipc = p->nnzC >= 0 && p->c_indptr_type == SPG_INDEX_32I ? 4 : 8;
    int64_t nnz = p->nnzC >= 0 ? p->nnzC : std::max<int64_t>(p->P, 0);
    *bytes = p->ws_bytes + ipc * (size_t)(p->A.rows + 1) +
             (size_t)nnz * (sizeof(int32_t) + vbytes(p->A.value_type));
    return SPG_STATUS_SUCCESS;
}

static spg_status_t check_cols16(const spg_csr_t* M, const void* starts, const void* lo16) {
    if (!M || M->rows < 0 || M->cols < 0 || M->nnz < 0) return SPG_STATUS_INVALID_VALUE;
    if (M->cols > 2147483647LL) return SPG_STATUS_NOT_SUPPORTED;
    if (M->indptr_type != SPG_INDEX_32I && M->indptr_type != SPG_INDEX_64I) return SPG_STATUS_INVALID_VALUE;
    if (!M->indptr) return SPG_STATUS_INVALID_VALUE;
    if (M->nnz > 0 && (!M->indices || !lo16)) return SPG_STATUS_INVALID_VALUE;
    if (M->cols > 65536 && M->rows > 0 && !starts) return SPG_STATUS_INVALID_VALUE;
    return SPG_STATUS_SUCCESS;
}

// interior block starts per row: ceil(cols / 65536) - 1 (none for a matrix <= 65536 wide)
static int cols16_nb1(const spg_csr_t* M) { return (int)std::max<int64_t>(0, (M->cols + 65535) / 65536 - 1); }

spg_status_t spg_cols16_split(spg_handle_t h, const spg_csr_t* M, uint32_t* block_starts, uint16_t* lo16) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    spg_status_t st = check_cols16(M, block_starts, lo16);
    if (st) return st;
    if (M->rows == 0) return SPG_STATUS_SUCCESS;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    const int nb1 = cols16_nb1(M);
    const dim3 g((unsigned)grid_for(M->rows, 4)), b(256);
    if (M->indptr_type == SPG_INDEX_64I)
        timed_launch(h, SPG_PHASE_LAYOUT, k_cols16_split<int64_t>, g, b, M->rows, (const int64_t*)M->indptr,
                     (const int32_t*)M->indices, nb1, block_starts, lo16);
    else
        timed_launch(h, SPG_PHASE_LAYOUT, k_cols16_split<int32_t>, g, b, M->rows, (const int32_t*)M->indptr,
                     (const int32_t*)M->indices, nb1, block_starts, lo16);
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_cols16_join(spg_handle_t h, spg_csr_t* M, const uint32_t* block_starts, const uint16_t* lo16) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    spg_status_t st = check_cols16(M, block_starts, lo16);
    if (st) return st;
    if (M->rows == 0) return SPG_STATUS_SUCCESS;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    const int nb1 = cols16_nb1(M);
    const dim3 g((unsigned)grid_for(M->rows, 4)), b(256);
    if (M->indptr_type == SPG_INDEX_64I)
        timed_launch(h, SPG_PHASE_LAYOUT, k_cols16_join<int64_t>, g, b, M->rows, (const int64_t*)M->indptr, nb1,
                     block_starts, lo16, (int32_t*)M->indices);
    else
        timed_launch(h, SPG_PHASE_LAYOUT, k_cols16_join<int32_t>, g, b, M->rows, (const int32_t*)M->indptr, nb1,
                     block_starts, lo16, (int32_t*)M->indices);
    SPG_LAUNCHED(h);
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_validate_csr(spg_handle_t h, const spg_csr_t* M, int* is_canonical) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!is_canonical) return SPG_STATUS_INVALID_VALUE;
    spg_status_t st = check_csr(M);
    if (st) return st;
    DeviceGuard dg_(h->device);
    SPG_HIP(h, dg_.err);
    if ((st = ensure_scratch(h, 256))) return st;
    int* flags = (int*)h->scratch;
    SPG_HIP(h, hipMemsetAsync(flags, 0, 2 * sizeof(int), h->stream));
    st = M->indptr_type == SPG_INDEX_64I ? validate_typed<int64_t>(h, *M, flags)
                                         : validate_typed<int32_t>(h, *M, flags);
    if (st) return st;
    SPG_HIP(h, hipMemcpyAsync(h->pinned, flags, 2 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    SPG_HIP(h, hipStreamSynchronize(h->stream));
    const int* f = (const int*)h->pinned;
    *is_canonical = f[1] ? -1 : (f[0] ? 0 : 1);
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_plan_info(spg_plan_t p, spg_plan_info_t* info, int64_t* chunk_rows, int64_t capacity) {
    if (!p || !info || capacity < 0 || (capacity > 0 && !chunk_rows)) return SPG_STATUS_INVALID_VALUE;
    info->path = p->use_tile ? 2 : (p->use_short ? 1 : 0);
    info->tile_width = p->use_tile ? (1 << p->tws) : 0;
    info->tiles_per_row = p->use_tile ? p->G : 0;
    info->record_group = p->use_tile ? (1 << p->rgs) : 0;
    info->dense_tiles = tile_dense(*p) ? 1 : 0;
    const bool chunked = p->alg == SPG_ALG3 && p->chunk_rows.size() > 1;
    info->n_chunks = chunked ? (int64_t)p->chunk_rows.size() - 1 : 1;
    // fp64 / complex128 tiles on the ordered-LDS kernels (k_tile_dn / k_tile_sp), or k_tile's
    // owner rounds (the handle's LDS check failed, or SPG_LDS_ORDERED=0)
    info->lds_ordered = p->use_tile && p->lean && (p->A.value_type == SPG_R_64F || p->A.value_type == SPG_C_64F) ? 1 : 0;
    for (int64_t i = 0; i < std::min<int64_t>(capacity, info->n_chunks + 1); ++i)
        chunk_rows[i] = chunked ? p->chunk_rows[(size_t)i] : (i == 0 ? 0 : p->A.rows);
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_plan_destroy(spg_plan_t p) {
    if (!p) return SPG_STATUS_INVALID_VALUE;
    delete p;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_spgemm_ws(spg_handle_t h, const spg_csr_t* A, const spg_csr_t* B, spg_alg_t alg,
                           float chunk_fraction, const void* alpha, void* workspace, size_t workspace_bytes,
                           void* C_indptr, spg_index_t C_indptr_type, int64_t* nnzC, void** C_indices,
                           void** C_values, size_t* peak_bytes, spg_plan_t* plan_out) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!alpha || !nnzC || !C_indices || !C_values || !peak_bytes || !plan_out) return SPG_STATUS_INVALID_VALUE;
    *plan_out = nullptr;
    *C_indices = *C_values = nullptr;
    spg_plan_t p = nullptr;
    size_t wsb = workspace_bytes;
    spg_status_t st = spg_plan(h, A, B, alg, chunk_fraction, &wsb, workspace, &p);
    if (st) return st;
    if ((st = spg_symbolic(h, p, C_indptr, C_indptr_type, nnzC))) {
        spg_plan_destroy(p);
        return st;
    }
    const size_t ipc = C_indptr_type == SPG_INDEX_32I ? 4 : 8;
    if (p->alg1_fused && *nnzC > 0) {
        // C already compact in the workspace: scale in place (alpha != 1) and finish
        spg_csr_t C{p->A.rows, p->B.cols, *nnzC, C_indptr, p->tj, p->tx, C_indptr_type, p->A.value_type};
        st = spg_numeric(h, p, alpha, &C);
        if (!st) {
            *C_indices = p->tj;
            *C_values = p->tx;
            *peak_bytes = p->ws_bytes + ipc * (size_t)(p->A.rows + 1);
        }
        spg_plan_destroy(p);
        return st;
    }
    *peak_bytes = p->ws_bytes + ipc * (size_t)(p->A.rows + 1) +
                  (size_t)*nnzC * (sizeof(int32_t) + vbytes(p->A.value_type));
    *plan_out = p;   // the caller allocates C's arrays, then spg_numeric + spg_plan_destroy
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_set_timing(spg_handle_t h, int enable) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    SPG_HIP(h, hipStreamSynchronize(h->stream));
    for (auto& q : h->pending) { h->pool.push_back(q.a); h->pool.push_back(q.b); }
    h->pending.clear();
    for (int i = 0; i < SPG_NUM_PHASES; ++i) { h->ms[i] = 0.0; h->launches[i] = 0; }
    h->timing = enable != 0;
    return SPG_STATUS_SUCCESS;
}

spg_status_t spg_get_timing(spg_handle_t h, spg_timing_t* t) {
    if (!h) return SPG_STATUS_NOT_INITIALIZED;
    if (!t) return SPG_STATUS_INVALID_VALUE;
    for (auto& q : h->pending) {
        SPG_HIP(h, hipEventSynchronize(q.b));
        float ms = 0.0f;
        SPG_HIP(h, hipEventElapsedTime(&ms, q.a, q.b));
        h->ms[q.phase] += ms;
        h->launches[q.phase] += 1;
        h->pool.push_back(q.a);
        h->pool.push_back(q.b);
    }
    h->pending.clear();
    for (int i = 0; i < SPG_NUM_PHASES; ++i) { t->ms[i] = h->ms[i]; t->launches[i] = h->launches[i]; }
    return SPG_STATUS_SUCCESS;
}

}  // extern "C"
