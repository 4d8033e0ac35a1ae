// sputnik-amd: host side of the sputnik::block API (C++ overloads) and its
// C-ABI twin (include/sputnik_amd.h).
//
// Replaces, for the hot path:
//   sputnik/block/dsd/dsd.cu:9-27, dds/dds.cu:7-24, sdd/sdd.cu:7-15
//     (block-size gate, Matmul/MatmulEx),
//   sputnik/block/{dsd,dds,sdd}/cutlass/<op>.cu (first-fit registries),
//   the can_launch_* / launch_* bodies of the 12 *_align8.cu variants
//     (shape rules, metadata checks, operand bundling),
//   sputnik/block/row_indices/row_indices.cu:24-36 and
//   sputnik/block/transpose/transpose.cu:69-125 (entry points).
//
// Problem -> kernel mapping (see block_gemm.h). Every product is phrased as
// O = S * D over 128-row tiles of a "row operand" S:
//   DSD  C = op(A) op(B):  S = op(A) (sparse), D = op(B), O = C.
//   DDS  C = op(A) op(B):  S = op(B)^T (sparse), D = op(A)^T, O = C^T.
//   SDD  C = op(A) op(B):  S = op(A) (dense),  D = op(B), O = C's blocks.
// A sparse S read in column order (DSD TN/TT, DDS NN/TN) uses the transposed
// metadata (offsets_t, indices_t, block_offsets), exactly like the reference.
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "api_internal.h"
#include "block_gemm.h"
#include "dsd4w.h"
#include "layout.h"
#include "metadata.h"
#include "sputnik/sputnik.h"
#include "sputnik_amd.h"

namespace sputnik_amd {

// Experiment builds (SPUTNIK_EXP & 128 / 512) copy this into
// GemmParams::debug.
static unsigned long long *g_debug = nullptr;

constexpr int kMaxDevices = 64;

// Compute units of a device, queried once per device (every SDD and every
// pair-eligible DSD/DDS call needs it).
static int DeviceCUs(int dev) {
  static int cached[kMaxDevices] = {};
  if (dev < 0 || dev >= kMaxDevices) return 0;
  int cus = __atomic_load_n(&cached[dev], __ATOMIC_RELAXED);
  if (cus > 0) return cus;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                            dev) != hipSuccess || cus <= 0)
    return 0;
  __atomic_store_n(&cached[dev], cus, __ATOMIC_RELAXED);
  return cus;
}

// ---- pair-balancing workspace ---------------------------------------------
// fp32 partial slots + hand-off flags + an error word, one set per (device,
// stream) so concurrent streams never share them. Allocated on the first
// eligible call and kept for the life of the process (like a BLAS handle's
// workspace). One workspace per stream relies on stream order: launches on
// one stream never overlap, so each launch owns the slots while it runs.
// Every launch carries a new epoch; a consumer waits for its own epoch, so a
// flag left by an earlier launch (or by a producer that published after its
// consumer gave up) can never satisfy a later launch, and nothing has to be
// reset. A launch captured into a graph replays one set of arguments and
// may replay on any stream, so captured launches get a workspace of their
// own per (device, capture, capturing stream) and keep their epoch on the
// device (GemmParams::pair_sync): replays of one graph are ordered behind
// each other, and no eager launch or other capture shares that workspace.
struct PairSlot {
  int device = -1;
  hipStream_t stream = nullptr;
  unsigned long long capture = 0;  // capture id (capture table only)
  // Capture table only: set (by a user-object destructor on HIP's callback
  // thread) once the captured graph and every executable made from it are
  // destroyed; the slot is then re-tied to the next capture that needs one
  // (PreparePairs / UseTall) or freed by sputnik_capture_workspaces().
  std::atomic<int> released{0};
  float *partials = nullptr;
  unsigned *flags = nullptr;  // [pairs] flags, the error word, [epoch, count]
  unsigned epoch = 0;
  int pairs = 0;  // capacity
  int slots = 0;  // resident workgroups on the device
};
constexpr int kMaxPairSlots = 16;
constexpr int kMaxCaptureSlots = 64;
static PairSlot g_pairs[kMaxPairSlots];
static PairSlot g_capture_pairs[kMaxCaptureSlots];
static std::mutex g_pairs_mu;

// ---- tuning knobs ---------------------------------------------------------
// Unsupported switches for same-process A/B experiments and tests (documented
// as such in include/sputnik_amd.h and INTEGRATION.md §6). Each starts from
// its environment variable, else its default, on first use; the C-ABI's
// sputnik_tuning_set() changes it at run time (process-wide). Defaults are
// the shipped configuration; nothing in a correct caller needs them.
struct KnobDef {
  const char *name;
  const char *env;
  int def, lo, hi;
};
static const KnobDef kKnobs[kNumKnobs] = {
    {"pairs", "SPUTNIK_AMD_PAIRS", 1, 0, 1},
    {"pair_xcd2", "SPUTNIK_AMD_PAIR_XCD2", 3, 0, 3},
    {"split", "SPUTNIK_AMD_SPLIT", 1, 0, 1},
    {"split_min_bn", "SPUTNIK_AMD_SPLIT_MIN_BN", 128, 0, 1 << 20},
    {"dsd4w", "SPUTNIK_AMD_DSD4W", 1, 0, 7},
    {"grouped_sdd", "SPUTNIK_AMD_GROUPED_SDD", 1, 0, 1},
    {"grouped_min_per_cu", "SPUTNIK_AMD_GROUPED_MIN_PER_CU", 4, 0, 1 << 20},
    {"tall", "SPUTNIK_AMD_TALL", 1, 0, 2},
    {"tall_persistent", "SPUTNIK_AMD_TALL_PERSISTENT", 1, 0, 1},
    {"dds_xcd2", "SPUTNIK_AMD_DDS_XCD2", 3, 0, 3},
    {"sdd4w_max_ld", "SPUTNIK_AMD_SDD4W_MAX_LD", 16384, 0, 1 << 30},
    {"pair_fault", "SPUTNIK_AMD_PAIR_FAULT", 0, 0, 1},
    // (off by default: every chunk of a K-split group waits for all of its
    // peers, so it needs the whole grid resident at once -- PrepareSddKsplit)
    {"sdd_ksplit", "SPUTNIK_AMD_SDD_KSPLIT", 1, 1, 8},
    {"sdd_ksplit_min_k", "SPUTNIK_AMD_SDD_KSPLIT_MIN_K", 6144, 512, 1 << 30},
    {"sdd_order", "SPUTNIK_AMD_SDD_ORDER", 1, 0, 4},
    {"tall4w", "SPUTNIK_AMD_TALL4W", 1, 0, 1},
    {"tall_flush_w", "SPUTNIK_AMD_TALL_FLUSH_W", 4, 0, 64},
    {"tall_odd_share", "SPUTNIK_AMD_TALL_ODD_SHARE", 120, 50, 200},
    {"min_handoff", "SPUTNIK_AMD_MIN_HANDOFF", 2, 1, 64},
    {"xcd_rows", "SPUTNIK_AMD_XCD_ROWS", 1, 0, 1},
    {"sdd_krot", "SPUTNIK_AMD_SDD_KROT", 0, 0, 4},
    // (2: NT only -- SDD NT 16384^3 dense 7603 -> 6934 us, config 4 in
    // MegaBlocks' w1 layout 812 -> 805 us, other NT shapes a tie; NN / TT
    // ties or noise, profiles/r06/ab/sdd_spread_ab.jsonl)
    {"sdd_spread", "SPUTNIK_AMD_SDD_SPREAD", 2, 0, 2},
    // (SDD NT / TT: B transposed first when its K N 2 bytes reach this many
    // MiB -- the MALL's 256 MB -- and the product is dense enough; 0 off)
    {"sdd_bt_min_mib", "SPUTNIK_AMD_SDD_BT_MIN_MIB", 256, 0, 1 << 20},
    // (grouped 4-wave SDD with K >= this: the rows past the groups' full
    // rounds go to an 8-wave launch of a block per workgroup; 0 off)
    {"sdd_tail_min_k", "SPUTNIK_AMD_SDD_TAIL_MIN_K", 8192, 0, 1 << 30},
};
constexpr int kKnobUnset = -0x7fffffff - 1;
static std::atomic<int> g_knobs[kNumKnobs];
static std::once_flag g_knobs_once;

static void InitKnobs() {
  std::call_once(g_knobs_once, [] {
    for (int i = 0; i < kNumKnobs; ++i) {
      const char *e = std::getenv(kKnobs[i].env);
      // (an unset, unparsable or out-of-range value means the default)
      char *end = nullptr;
      const long v0 = e != nullptr && *e != 0 ? std::strtol(e, &end, 10) : 0;
      const bool ok = e != nullptr && *e != 0 && end != nullptr && *end == 0 &&
                      v0 >= kKnobs[i].lo && v0 <= kKnobs[i].hi;
      const int v = ok ? (int)v0 : kKnobs[i].def;
      g_knobs[i].store(v, std::memory_order_relaxed);
    }
  });
}

int Knob(KnobId k) {
  InitKnobs();
  return g_knobs[k].load(std::memory_order_relaxed);
}

static int KnobIndex(const char *name) {
  if (name == nullptr) return -1;
  for (int i = 0; i < kNumKnobs; ++i)
    if (std::strcmp(name, kKnobs[i].name) == 0) return i;
  return -1;
}

int TuningGet(const char *name) {
  const int i = KnobIndex(name);
  return i < 0 ? kKnobUnset : Knob(static_cast<KnobId>(i));
}

int TuningSet(const char *name, int value) {
  const int i = KnobIndex(name);
  if (i < 0 || value < kKnobs[i].lo || value > kKnobs[i].hi) return kKnobUnset;
  InitKnobs();
  return g_knobs[i].exchange(value, std::memory_order_relaxed);
}

// Tile counter pair of persistent tall launches, per (device, stream): the
// kernel resets it to zero at the end of every launch (GemmParams::
// tile_counter), so launches on one stream need no host-side bookkeeping.
// Not used under graph capture (a replay on another stream could overlap an
// eager launch on this one) nor on hipStreamPerThread, whose one handle
// stands for many concurrently running streams.
struct CounterSlot {
  int device = -1;
  hipStream_t stream = nullptr;
  unsigned long long capture = 0;  // capture id (capture table only)
  std::atomic<int> released{0};  // as PairSlot::released
  unsigned long long *counter = nullptr;  // [fetch, done]
};
static CounterSlot g_counters[kMaxPairSlots];
static CounterSlot g_capture_counters[kMaxCaptureSlots];

// Capture status of `stream`: 0 not capturing, 1 capturing (id in *id),
// -1 the query failed or the capture is invalidated (no workspace then).
static int CaptureState(hipStream_t stream, unsigned long long *id) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  *id = 0;
  if (hipStreamGetCaptureInfo(stream, &cs, id) != hipSuccess) return -1;
  if (cs == hipStreamCaptureStatusNone) return 0;
  return cs == hipStreamCaptureStatusActive ? 1 : -1;
}

// Device memory for a workspace, zero-filled, callable while `stream` is
// being captured: the thread switches to relaxed capture mode (hipMalloc is
// not a stream operation), and the fill runs on a private non-blocking
// stream that no capture touches, synchronized before returning.
// The library's private non-blocking stream of a device (created on first
// use, kept for the process; caller holds g_pairs_mu).
static hipStream_t g_side[kMaxDevices] = {};
static hipError_t SideStream(int dev, hipStream_t *out) {
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  if (g_side[dev] == nullptr) {
    const hipError_t e = hipStreamCreateWithFlags(&g_side[dev], hipStreamNonBlocking);
    if (e != hipSuccess) return e;
  }
  *out = g_side[dev];
  return hipSuccess;
}

static hipError_t AllocZeroed(void **ptr, size_t bytes, int dev) {
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  hipStream_t side = nullptr;
  hipError_t e = SideStream(dev, &side);
  *ptr = nullptr;
  if (e == hipSuccess) e = hipMalloc(ptr, bytes);
  if (e == hipSuccess) e = hipMemsetAsync(*ptr, 0, bytes, side);
  if (e == hipSuccess) e = hipStreamSynchronize(side);
  if (e != hipSuccess && *ptr != nullptr) {
    (void)hipFree(*ptr);
    *ptr = nullptr;
  }
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  return e;
}

// Ties a capture-table slot to the lifetime of the graph being captured on
// `stream`: a user object retained by the graph (executables instantiated
// from it retain it too) sets *released when the last reference goes, i.e.
// once the graph and all its executables are destroyed and no launch of them
// is pending. A destructor may not call HIP, so the memory is freed later by
// ReclaimCaptureSlots. Returns false if the graph cannot be tied (the slot
// then lives for the process, as before).
static void MarkReleased(void *flag) {
  static_cast<std::atomic<int> *>(flag)->store(1, std::memory_order_release);
}
static bool TieToCapturedGraph(hipStream_t stream, std::atomic<int> *released) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t *deps = nullptr;
  size_t ndeps = 0;
  if (hipStreamGetCaptureInfo_v2(stream, &cs, &id, &graph, &deps, &ndeps) !=
          hipSuccess ||
      cs != hipStreamCaptureStatusActive || graph == nullptr)
    return false;
  hipUserObject_t obj = nullptr;
  if (hipUserObjectCreate(&obj, released, MarkReleased, 1,
                          hipUserObjectNoDestructorSync) != hipSuccess)
    return false;
  // Move our one reference into the graph: the graph now owns the object.
  if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) !=
      hipSuccess) {
    (void)hipUserObjectRelease(obj, 1);
    return false;
  }
  return true;
}

// Frees the capture-table workspaces whose graphs are gone (caller holds
// g_pairs_mu; called from eager launches only, never while this thread's
// stream is being captured, since hipFree is not a capturable call).
static void FreeQuiet(void *ptr) {
  if (ptr == nullptr) return;
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipFree(ptr);
  (void)hipThreadExchangeStreamCaptureMode(&mode);
}
static void ReclaimCaptureSlots();

// A (device, stream) table ran out of slots: the caller falls back to the
// plain launch (correct, slower); said once per process.
// kind: 0 pair balancing, 1 persistent launches; +2 in captured graphs.
static void WarnSlotsFull(int kind) {
  static bool warned[4] = {false, false, false, false};
  static const char *const what[4] = {
      "streams use pair balancing", "streams use persistent launches",
      "graph captures use pair balancing",
      "graph captures use persistent launches"};
  if (kind >= 0 && kind < 4 && !warned[kind]) {
    warned[kind] = true;
    SPUTNIK_LOG(WARNING) << "sputnik-amd: more than "
                         << (kind < 2 ? kMaxPairSlots : kMaxCaptureSlots)
                         << " " << what[kind]
                         << "; further ones run without it";
  }
}

static bool PairsEnabled() {
#ifdef SPUTNIK_NO_PAIRS
  return false;
#endif
  return Knob(kKnobPairs) != 0;
}

// Fills the pair fields of p when pair balancing applies: a staggered
// one-workgroup-per-CU tile config, every tile resident at once (the point
// is the tail of a single wave of tiles) and rows rankable in-kernel. Below
// a mean of 2 blocks per row the hand-offs cost more than the tail they
// shorten (DSD 4096² at 5%: 23.7 µs with pairs, 20.3 µs without; unchanged
// from 7% up, same-process A/B r01l).
#ifndef SPUTNIK_PAIR_MIN_MEAN4
#define SPUTNIK_PAIR_MIN_MEAN4 8  // 4 x mean blocks per row
#endif
// dry: decide only (DsdPlan): no workspace is allocated, re-tied or
// advanced, and the pointers stay null.
// The pair workspace of (device, stream) -- or of the capture under way on
// `stream` -- found, re-tied or allocated (caller holds g_pairs_mu). dry:
// decide only; a slot that would be allocated is described in *dry_slot
// and nothing is allocated, re-tied or advanced. nullptr: none available.
static PairSlot *AcquirePairSlot(hipStream_t stream, bool dry, PairSlot *dry_slot,
                                 int *capturing_out) {
  unsigned long long capture = 0;
  const int capturing = CaptureState(stream, &capture);
  *capturing_out = capturing;
  if (capturing < 0) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  PairSlot *table = capturing ? g_capture_pairs : g_pairs;
  const int n_table = capturing ? kMaxCaptureSlots : kMaxPairSlots;
  for (int i = 0; i < n_table; ++i) {
    PairSlot &s = table[i];
    if (s.partials != nullptr && s.device == dev && s.stream == stream &&
        s.capture == capture)
      return &s;
  }
  // A capture-table slot whose graph is gone is re-tied to the graph being
  // captured, memory and device epoch word as they are: the word only ever
  // grows, so the flags the old graph left can never match a new launch, and
  // its arrival count is back at zero (the last arriver of every launch
  // resets it). No HIP free on this path (frees happen in
  // sputnik_capture_workspaces()).
  if (capturing) {
    for (int i = 0; i < n_table; ++i) {
      PairSlot &s = table[i];
      if (s.partials != nullptr && s.device == dev &&
          s.released.load(std::memory_order_acquire) != 0) {
        if (dry) return &s;
        s.stream = stream;
        s.capture = capture;
        s.released.store(0, std::memory_order_relaxed);
        (void)TieToCapturedGraph(stream, &s.released);
        return &s;
      }
    }
  }
  PairSlot *slot = nullptr;
  for (int i = 0; i < n_table; ++i)
    if (table[i].partials == nullptr) {
      slot = &table[i];
      break;
    }
  if (slot == nullptr) {
    if (!dry) WarnSlotsFull(capturing ? 2 : 0);
    return nullptr;
  }
  const int cus = DeviceCUs(dev);
  if (cus <= 0) return nullptr;
  const int slots = cus * CfgSparse::kWGs;
  // Partial slots of 128 x 512 fp32 (256 KiB): one per resident workgroup
  // (a pair uses one per pair, split mode one per tile, the SDD K-split one
  // per workgroup): 64 MiB per workspace on MI355X. Flags: [pairs] pair
  // flags, the error word, [epoch, count] (pair_sync), [slots] K-split flags.
  const int pairs = slots / 2;
  if (dry) {  // the workspace a launch would allocate
    dry_slot->slots = slots;
    dry_slot->pairs = pairs;
    return dry_slot;
  }
  void *partials = nullptr, *flags = nullptr;
  if (AllocZeroed(&partials, (size_t)slots * kBM * CfgSparse::kBN * sizeof(float), dev) !=
      hipSuccess)
    return nullptr;
  if (AllocZeroed(&flags, (pairs + 3 + slots) * sizeof(unsigned), dev) != hipSuccess) {
    FreeQuiet(partials);
    return nullptr;
  }
  slot->device = dev;
  slot->stream = stream;
  slot->capture = capture;
  slot->partials = static_cast<float *>(partials);
  slot->flags = static_cast<unsigned *>(flags);
  slot->pairs = pairs;
  slot->slots = slots;
  slot->released.store(0, std::memory_order_relaxed);
  if (capturing) (void)TieToCapturedGraph(stream, &slot->released);
  return slot;
}

// A new epoch and the workspace pointers for one launch.
static void BindPairSlot(GemmParams *p, PairSlot *slot, int capturing) {
  if (++slot->epoch == 0) slot->epoch = 1;  // 0 is the initial flag value
  p->pair_partials = slot->partials;
  p->pair_flags = slot->flags;
  p->pair_epoch = slot->epoch;
  p->pair_error = slot->flags + slot->pairs;
  p->pair_sync = capturing ? slot->flags + slot->pairs + 1 : nullptr;
  p->ks_flags = slot->flags + slot->pairs + 3;
}

static void PreparePairs(GemmParams *p, long long blocks, hipStream_t stream,
                         bool dry = false) {
  p->pair = 0;
  if (!CfgSparse::kStagger || CfgSparse::kWGs != 1)
    return;
  if (!PairsEnabled() || p->num_rows < 2 || p->num_rows > kLptRows) return;
  if (blocks * 4 < (long long)p->num_rows * SPUTNIK_PAIR_MIN_MEAN4) return;
  if (stream == hipStreamPerThread) return;  // many streams, one handle
  std::lock_guard<std::mutex> lock(g_pairs_mu);
  PairSlot dry_slot;
  int capturing = 0;
  PairSlot *slot = AcquirePairSlot(stream, dry, &dry_slot, &capturing);
  if (slot == nullptr) return;
  if (p->num_tiles > slot->slots) return;
  p->pair = 1;
  if (!dry) BindPairSlot(p, slot, capturing);
  p->pair_fault = Knob(kKnobPairFault);
  // Two panels x half the pairs per XCD (GemmParams::pair_xcd2) from a mean
  // of 8 blocks per row: DSD 4096^3 A/B (r02m) 30% / 50% / 90% +1.2 / +2.7
  // / +2.8%, 10% -4.4%. SPUTNIK_AMD_PAIR_XCD2=0 turns it off. Mode 3 (the
  // default) gives the heavy half of the pairs (the ones with hand-offs) to
  // the odd XCD of each panel pair: per-workgroup timelines (r04f/g,
  // scripts/exp_timeline4w.py) show logical XCDs 0/2/4/6 running the same
  // k-loop ~6% slower per block than 1/3/7 on every box measured, and mode
  // 1 had put the critical pairs exactly there (4-wave A/B, separate
  // processes, 30/50/90%: +1.0/+2.1/+1.4%, 10% +0.5%). Mode 2 interleaves
  // the pairs (r04d: +0.5% at 50%).
  const int xcd2 = Knob(kKnobPairXcd2);
  p->pair_xcd2 = xcd2 != 0 && blocks >= 8LL * p->num_rows ? xcd2 : 0;
  p->min_handoff = Knob(kKnobMinHandoff);
  // Split mode (GemmParams::pair_split) when the tiles fill at most half of
  // the workgroup slots (e.g. 512-2048-row panels of a strong-scaled 4096^2,
  // or narrow N) and the rows hold at least 4 blocks on average: two
  // workgroups per tile. SPUTNIK_AMD_SPLIT=0 turns it off. (r03b, DSD
  // K=N=4096 50%: M=512 45.2 -> 34.6 us, 1024 47.6 -> 38.4, 2048 48.8 ->
  // 45.2; 4 or 8 workgroups per tile were slower.)
  const int split_on = Knob(kKnobSplit);
  // Tile width: the narrowest of 512 / 256 / 128 columns whose tiles (two
  // workgroups each) still fit the slots, so a panel of few block-rows
  // fills the CUs (r03: M = 512 on 128-column tiles, M = 1024 on 256).
  int split = 1;
  if (split_on != 0 && (long long)p->num_tiles * 2 <= slot->slots &&
      blocks >= 4LL * p->num_rows) {
    split = 2;
    int bn = CfgSparse::kBN;
    for (int cand : {256, 128}) {
      const long long tiles =
          (long long)p->num_rows * ((p->j_limit + cand - 1) / cand);
      if (tiles * 2 > slot->slots) break;
      bn = cand;
    }
    // Tuning floor of the tile width: 512 keeps the wide tile. Only the
    // three instantiated widths are valid (Launch has split kernels for 128,
    // 256 and 512 columns); anything else is rounded up to the next one.
    const int mbn = Knob(kKnobSplitMinBn);
    const int max_narrow = mbn <= 128 ? 128 : mbn <= 256 ? 256 : CfgSparse::kBN;
    if (bn < max_narrow) bn = max_narrow;
    p->split_bn = bn;
    p->num_jtiles = (p->j_limit + bn - 1) / bn;
    p->num_tiles = p->num_rows * p->num_jtiles;
  }
  p->pair_split = split;
  if (split > 1) p->grid = split * p->num_tiles;
}

// Pair hand-offs that timed out (and were recomputed by their consumer)
// since the last call, summed over every workspace of the current device;
// the error words are cleared. One device-wide
// synchronize first: the streams the workspaces were made for may have been
// destroyed since (or their handles reused), so they are never used here.
int PairErrors() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  std::lock_guard<std::mutex> lock(g_pairs_mu);
  int total = 0;
  for (int i = 0; i < kMaxPairSlots + kMaxCaptureSlots; ++i) {
    PairSlot &s = i < kMaxPairSlots ? g_pairs[i]
                                    : g_capture_pairs[i - kMaxPairSlots];
    if (s.partials == nullptr || s.device != dev) continue;
    unsigned word = 0;
    if (hipMemcpy(&word, s.flags + s.pairs, sizeof(word),
                  hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    if (word != 0) {
      total += (int)word;
      const unsigned zero = 0;
      if (hipMemcpy(s.flags + s.pairs, &zero, sizeof(zero),
                    hipMemcpyHostToDevice) != hipSuccess)
        return -1;
    }
  }
  return total;
}

void SetPairFault(int on) { (void)TuningSet("pair_fault", on != 0 ? 1 : 0); }

// DSD NN kernel selection: the 4-wave hand-scheduled kernel (dsd4w.hip) where
// it applies, else the 8-wave block_gemm_kernel. Knob "dsd4w" 0 (tests and
// A/B) keeps the 8-wave kernel.
static int Dsd4wMode() { return Knob(kKnobDsd4w); }
bool Dsd4wEnabled() { return Dsd4wMode() != 0; }
// 2..7: wherever the kernel can run, whatever the density (tests, A/B), with
// epilogue 0 .. 5 (dsd4w.h LaunchDsd4w); 1: the default epilogue.
bool Dsd4wForced() { return Dsd4wMode() >= 2; }
int Dsd4wEpi() {
  const int m = Dsd4wMode();
  return m >= 2 ? m - 2 : kDsd4wDefaultEpi;
}
int SelectDsdKernel(int four_wave) {
  if (four_wave < 0) return Dsd4wMode();
  return TuningSet("dsd4w", four_wave > 7 ? 7 : four_wave);
}

static void ReclaimCaptureSlots() {
  for (auto &sl : g_capture_pairs) {
    if (sl.partials == nullptr ||
        sl.released.load(std::memory_order_acquire) == 0)
      continue;
    FreeQuiet(sl.partials);
    FreeQuiet(sl.flags);
    sl.partials = nullptr;
    sl.flags = nullptr;
    sl.device = -1;
    sl.stream = nullptr;
    sl.capture = 0;
    sl.epoch = 0;
    sl.pairs = sl.slots = 0;
    sl.released.store(0, std::memory_order_relaxed);
  }
  for (auto &c : g_capture_counters) {
    if (c.counter == nullptr || c.released.load(std::memory_order_acquire) == 0)
      continue;
    FreeQuiet(c.counter);
    c.counter = nullptr;
    c.device = -1;
    c.stream = nullptr;
    c.capture = 0;
    c.released.store(0, std::memory_order_relaxed);
  }
}

int CaptureWorkspaces() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> lock(g_pairs_mu);
  ReclaimCaptureSlots();
  int n = 0;
  for (const auto &s : g_capture_pairs)
    n += s.partials != nullptr && s.device == dev;
  for (const auto &c : g_capture_counters)
    n += c.counter != nullptr && c.device == dev;
  return n;
}

namespace {

using sputnik::block::AsInt;
using sputnik::block::BlockSize;
using sputnik::block::MatmulShape;
using sputnik::block::ValidMatmul;

constexpr long long kMaxLaneOffset = 0x7fffffffLL;  // 31-bit buffer offsets

bool DenseOk(const Matrix &m) {
  return m.rows >= 0 && m.cols >= 0 &&
         (m.data != nullptr || (long long)m.rows * m.cols == 0);
}

bool SparseOk(const BlockMatrix &s) {
  const int b = AsInt(s.block_size);
  if (b != 128) return false;
  if (s.rows < 0 || s.cols < 0 || s.nonzeros < 0) return false;
  if (s.rows % b != 0 || s.cols % b != 0 || s.nonzeros % (b * b) != 0)
    return false;
  if ((s.cols / b) > 32767 || (s.rows / b) > 32767) return false;  // int16
  if (s.offsets == nullptr) return false;
  if (s.nonzeros > 0 && (s.data == nullptr || s.indices == nullptr))
    return false;
  return true;
}

// The reference's BlockGemm::can_implement: m, n, k multiples of 8
// (block_gemm.h:728-745; 8 x fp16 = one 16-byte access).
bool Aligned8(const MatmulShape &s) {
  return s.m % 8 == 0 && s.n % 8 == 0 && s.k % 8 == 0 && s.m >= 0 &&
         s.n >= 0 && s.k >= 0;
}

// Rows of one DMA tile times the byte stride must fit a 31-bit lane offset.
bool StrideOk(long long rows_in_tile, long long ld_elems) {
  return rows_in_tile * ld_elems * 2 <= kMaxLaneOffset;
}

Status PrepareDsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const Matrix &c, GemmParams *p, bool *needs_meta) {
  if (a.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(a) || !DenseOk(b) || !DenseOk(c)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s)) return Status::kNoKernel;
  const bool d_kc = tb;  // B^T stored [N][K]: k-contiguous
  if (!StrideOk(d_kc ? CfgSparse::kBN : 64, s.ldb)) return Status::kNoKernel;
  *needs_meta = ta;
  if (ta && (a.offsets_t == nullptr || a.indices_t == nullptr ||
             a.block_offsets == nullptr))
    return Status::kMissingMetadata;

  *p = GemmParams{};
  p->s_data = static_cast<const char *>(a.data);
  p->s_offsets = static_cast<const int *>(ta ? a.offsets_t : a.offsets);
  p->s_indices = static_cast<const short *>(ta ? a.indices_t : a.indices);
  p->s_block_offsets =
      ta ? static_cast<const int *>(a.block_offsets) : nullptr;
  p->s_blocks = (int)(a.nonzeros / (kBlock * kBlock));
  p->d_data = static_cast<const char *>(b.data);
  p->d_ld = (long long)s.ldb * 2;
  p->c_data = static_cast<char *>(c.data);
  p->c_ld = (long long)s.ldc * 2;
  p->num_rows = s.m / kBM;
  p->num_jtiles = (s.n + CfgSparse::kBN - 1) / CfgSparse::kBN;
  p->j_limit = s.n;
  p->num_tiles = p->num_rows * p->num_jtiles;
  return Status::kOk;
}

Status PrepareDds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const Matrix &c, GemmParams *p, bool *needs_meta) {
  if (b.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(b) || !DenseOk(a) || !DenseOk(c)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s)) return Status::kNoKernel;
  const bool d_kc = !ta;  // op(A)^T rows are A's rows when A is [M][K]
  if (!StrideOk(d_kc ? CfgSparse::kBN : 64, s.lda)) return Status::kNoKernel;
  // Row n of op(B)^T is column n of B when B is stored [K][N] (tb == false).
  const bool col_order = !tb;
  *needs_meta = col_order;
  if (col_order && (b.offsets_t == nullptr || b.indices_t == nullptr ||
                    b.block_offsets == nullptr))
    return Status::kMissingMetadata;

  *p = GemmParams{};
  p->s_data = static_cast<const char *>(b.data);
  p->s_offsets = static_cast<const int *>(col_order ? b.offsets_t : b.offsets);
  p->s_indices =
      static_cast<const short *>(col_order ? b.indices_t : b.indices);
  p->s_block_offsets =
      col_order ? static_cast<const int *>(b.block_offsets) : nullptr;
  p->d_data = static_cast<const char *>(a.data);
  p->d_ld = (long long)s.lda * 2;
  p->c_data = static_cast<char *>(c.data);
  p->c_ld = (long long)s.ldc * 2;
  p->s_blocks = (int)(b.nonzeros / (kBlock * kBlock));
  p->num_rows = s.n / kBM;
  p->num_jtiles = (s.m + CfgSparse::kBN - 1) / CfgSparse::kBN;
  p->j_limit = s.m;
  p->num_tiles = p->num_rows * p->num_jtiles;
  return Status::kOk;
}

Status PrepareSdd(const Matrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, GemmParams *p) {
  if (c.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(c) || !DenseOk(a) || !DenseOk(b)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s)) return Status::kNoKernel;
  if (!StrideOk(ta ? 64 : 128, s.lda) || !StrideOk(tb ? 128 : 64, s.ldb))
    return Status::kNoKernel;
  const int blocks = c.nonzeros / (kBlock * kBlock);
  if (blocks > 0 && c.row_indices == nullptr)
    return Status::kMissingRowIndices;

  *p = GemmParams{};
  p->s_data = static_cast<const char *>(a.data);
  p->s_ld = (long long)s.lda * 2;
  p->d_data = static_cast<const char *>(b.data);
  p->d_ld = (long long)s.ldb * 2;
  p->c_data = static_cast<char *>(c.data);
  p->c_row_indices = static_cast<const short *>(c.row_indices);
  p->c_indices = static_cast<const short *>(c.indices);
  p->num_rows = s.m / kBM;
  p->j_limit = s.n;
  p->k_limit = s.k;
  p->num_tiles = blocks;
  return Status::kOk;
}

// SSD / SDS: a sparse operand as in DSD / DDS, a sparse output as in SDD
// (reference ssd.cu:7-24 and sds.cu:7-24; their *_align8.cu variants need
// the sparse input's transposed metadata exactly where DSD / DDS do, and
// c.row_indices always).
Status PrepareSparseOut(const BlockMatrix &c, GemmParams *p) {
  if (c.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(c)) return Status::kNoKernel;
  const int blocks = c.nonzeros / (kBlock * kBlock);
  if (blocks > 0 && c.row_indices == nullptr)
    return Status::kMissingRowIndices;
  p->c_data = static_cast<char *>(c.data);
  p->c_row_indices = static_cast<const short *>(c.row_indices);
  p->c_indices = static_cast<const short *>(c.indices);
  p->num_tiles = blocks;
  return Status::kOk;
}

Status PrepareSsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, GemmParams *p, bool *needs_meta) {
  if (a.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(a) || !DenseOk(b)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s)) return Status::kNoKernel;
  if (!StrideOk(tb ? kBlock : 64, s.ldb)) return Status::kNoKernel;
  *needs_meta = ta;
  if (ta && (a.offsets_t == nullptr || a.indices_t == nullptr ||
             a.block_offsets == nullptr))
    return Status::kMissingMetadata;
  *p = GemmParams{};
  const Status st = PrepareSparseOut(c, p);
  if (st != Status::kOk) return st;
  p->s_data = static_cast<const char *>(a.data);
  p->s_offsets = static_cast<const int *>(ta ? a.offsets_t : a.offsets);
  p->s_indices = static_cast<const short *>(ta ? a.indices_t : a.indices);
  p->s_block_offsets =
      ta ? static_cast<const int *>(a.block_offsets) : nullptr;
  p->d_data = static_cast<const char *>(b.data);
  p->d_ld = (long long)s.ldb * 2;
  p->num_rows = s.m / kBM;
  p->j_limit = s.n;
  return Status::kOk;
}

Status PrepareSds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const BlockMatrix &c, GemmParams *p, bool *needs_meta) {
  if (b.block_size != BlockSize::k128) return Status::kNotSupported;
  if (!SparseOk(b) || !DenseOk(a)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s)) return Status::kNoKernel;
  if (!StrideOk(!ta ? kBlock : 64, s.lda)) return Status::kNoKernel;
  const bool col_order = !tb;
  *needs_meta = col_order;
  if (col_order && (b.offsets_t == nullptr || b.indices_t == nullptr ||
                    b.block_offsets == nullptr))
    return Status::kMissingMetadata;
  *p = GemmParams{};
  const Status st = PrepareSparseOut(c, p);
  if (st != Status::kOk) return st;
  p->s_data = static_cast<const char *>(b.data);
  p->s_offsets = static_cast<const int *>(col_order ? b.offsets_t : b.offsets);
  p->s_indices =
      static_cast<const short *>(col_order ? b.indices_t : b.indices);
  p->s_block_offsets =
      col_order ? static_cast<const int *>(b.block_offsets) : nullptr;
  p->d_data = static_cast<const char *>(a.data);
  p->d_ld = (long long)s.lda * 2;
  p->num_rows = s.n / kBM;
  p->j_limit = s.m;
  return Status::kOk;
}

// DSS: C = op(A_bcsr) op(B_bcsr), dense (reference dss.cu:9-24). op(A)'s
// rows use A's transposed metadata when transpose_a; op(B)'s columns use B's
// transposed metadata unless transpose_b (dss_*_align8.cu). K <= 32768
// (dss_nn:67). The reference's bitmask workspaces are not needed: the
// intersection is built per tile in LDS.
constexpr int kDssMaxK = 32768;
Status PrepareDss(const BlockMatrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const Matrix &c, GemmParams *p, bool *meta_a,
                  bool *meta_b) {
  if (a.block_size != BlockSize::k128 || b.block_size != BlockSize::k128)
    return Status::kNotSupported;
  if (!SparseOk(a) || !SparseOk(b) || !DenseOk(c)) return Status::kNoKernel;
  if (!ValidMatmul(a, ta, b, tb, c)) return Status::kNoKernel;
  const MatmulShape s(a, ta, b, tb);
  if (!Aligned8(s) || s.k > kDssMaxK) return Status::kNoKernel;
  *meta_a = ta;
  *meta_b = !tb;
  if (ta && (a.offsets_t == nullptr || a.indices_t == nullptr ||
             a.block_offsets == nullptr))
    return Status::kMissingMetadata;
  if (!tb && (b.offsets_t == nullptr || b.indices_t == nullptr ||
              b.block_offsets == nullptr))
    return Status::kMissingMetadata;
  *p = GemmParams{};
  p->s_data = static_cast<const char *>(a.data);
  p->s_offsets = static_cast<const int *>(ta ? a.offsets_t : a.offsets);
  p->s_indices = static_cast<const short *>(ta ? a.indices_t : a.indices);
  p->s_block_offsets =
      ta ? static_cast<const int *>(a.block_offsets) : nullptr;
  p->d_data = static_cast<const char *>(b.data);
  p->d_ld = kBlock * 2;  // inside one stored 128x128 block
  p->d_offsets = static_cast<const int *>(tb ? b.offsets : b.offsets_t);
  p->d_indices = static_cast<const short *>(tb ? b.indices : b.indices_t);
  p->d_block_offsets =
      tb ? nullptr : static_cast<const int *>(b.block_offsets);
  p->c_data = static_cast<char *>(c.data);
  p->c_ld = (long long)s.ldc * 2;
  p->num_rows = s.m / kBM;
  p->num_jtiles = s.n / kBlock;
  p->j_limit = s.n;
  p->num_tiles = p->num_rows * p->num_jtiles;
  return Status::kOk;
}

hipError_t BuildTransposed(const BlockMatrix &a, hipStream_t stream) {
  const int b = AsInt(a.block_size);
  if (b == 0) return hipErrorNotSupported;
  return LaunchTransposeMetadata(
      a.rows / b, a.cols / b, static_cast<int>(a.nonzeros / (b * b)),
      static_cast<const int *>(a.offsets),
      static_cast<const short *>(a.indices), static_cast<int *>(a.offsets_t),
      static_cast<short *>(a.indices_t), static_cast<int *>(a.block_offsets),
      stream);
}

// C++ API convention: abort where the reference aborts.
hipError_t OrAbort(Status st, const char *op) {
  switch (st) {
    case Status::kOk: return hipSuccess;
    case Status::kNotSupported: return hipErrorNotSupported;
    case Status::kNoKernel:
      SPUTNIK_LOG(FATAL) << "No compatible kernel for " << op << " problem.";
      break;
    case Status::kMissingMetadata:
      SPUTNIK_LOG(FATAL) << "Check failed: offsets_t && indices_t && "
                            "block_offsets (" << op << ")";
      break;
    case Status::kMissingRowIndices:
      SPUTNIK_LOG(FATAL) << "Check failed: c.row_indices (" << op << ")";
      break;
  }
  return hipErrorUnknown;
}

// C-ABI convention: never abort.
int AsCode(Status st) {
  switch (st) {
    case Status::kOk: return hipSuccess;
    case Status::kNotSupported: return hipErrorNotSupported;
    default: return hipErrorInvalidValue;
  }
}

// Grouped SDD tiles (CfgSddGrouped: up to 4 stored blocks of a block-row per
// workgroup) when there are enough groups to fill the CUs, the rows fit the
// in-kernel group scan, and every gathered D offset fits the 31-bit lane
// offset. Sets the grid to the upper bound nb/4 + rows; surplus workgroups
// exit at once.
constexpr int kMaxGroupRows = 32767;
bool UseGroupedSdd(GemmParams *p, const BlockMatrix &c, bool d_kc) {
#ifdef SPUTNIK_NO_GROUPED_SDD
  return false;
#endif
  if (Knob(kKnobGroupedSdd) == 0 || c.offsets == nullptr) return false;
  constexpr int kGrp = CfgSddGrouped::kBN / kBlock;
  const int blocks = p->num_tiles;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const int cus = DeviceCUs(dev);
  if (cus <= 0) return false;
  // From 4 blocks per CU the grouped tile is faster: the 4-wave grouped
  // kernel with its groups mapped over the actual group count (r05 gm2,
  // same process: SDD 4096^3 dense = 4 per CU, every transpose 100-103 us
  // vs 158-164 us on the k-split tile; 2 per CU 77 vs 76, 3.2 per CU 286 vs
  // 286: tie). r02's 8-wave grouped tile needed 5 per CU (scripts/
  // exp_grp.sh: 4 per CU k-split 318 vs grouped 362 us, 5 per CU 399 vs 365).
  // Knob "grouped_min_per_cu" (default 4) moves the switch (tuning only;
  // never below kGrp, so a grouped grid still fills every CU).
  static_assert(4 >= kGrp, "a grouped grid fills every CU");
  const int min_per_cu = Knob(kKnobGroupedMinPerCu) < kGrp ? kGrp
                                                             : Knob(kKnobGroupedMinPerCu);
  if (blocks < min_per_cu * cus || p->num_rows > kMaxGroupRows)
    return false;
  // D lane offsets: k-contiguous D gathers whole rows (n * ldb); otherwise
  // one 32-row k panel plus any column.
  const long long span = d_kc ? (long long)p->j_limit * p->d_ld
                              : 32LL * p->d_ld + (long long)p->j_limit * 2;
  if (span > kMaxLaneOffset) return false;
  p->c_offsets = static_cast<const int *>(c.offsets);
  p->num_tiles = blocks / kGrp + p->num_rows + 1;
  return true;
}

// SDD NN with too few stored blocks for the grouped grid (UseGroupedSdd
// false) and few enough groups that every group can take 2 or more
// workgroups: the 4-wave grouped kernel with each group's K split over S in
// {2, 4, 8} workgroups (GemmParams::sdd_ksplit, S chosen in-kernel from the
// actual group count), the partials reduced through the pair workspace.
// Grid = one workgroup per CU, all resident at once (one 160-KiB-LDS
// workgroup fits a CU): every chunk of a group is running while its peers
// wait for it. That all-to-all wait is why it is OFF by default (knob
// sdd_ksplit = 1): a launch that shares the device with another
// kernel holding CUs for longer than the 0.2 s bounded wait (an RCCL kernel
// on a side stream, a CU-masked stream) would leave chunks undispatched
// while their peers time out, and the launch would return NaN tiles (counted
// by sputnik_pair_errors()). Unlike the DSD pair hand-off -- a consumer waits
// only on a producer dispatched before it -- no chunk order avoids this, and
// a last-arriver reduction would serialize S - 1 partials on one CU (the
// gain at K = 8192 was 5%). Opt in with sputnik_tuning_set("sdd_ksplit", 8)
// when the launch has the device to itself.
// dry: decide only (SddPlan), no workspace allocated, re-tied or advanced.
static bool PrepareSddKsplit(GemmParams *p, const BlockMatrix &c, bool ta, bool tb,
                             hipStream_t stream, bool dry = false) {
  const int max_s = Knob(kKnobSddKsplit);
  if (max_s < 2 || ta || tb || c.offsets == nullptr || !Dsd4wEnabled()) return false;
  // From K = 6144 (knob sdd_ksplit_min_k): its fixed cost -- every chunk
  // publishes (S - 1) / S of its fp32 tile and reads as much back, ~10 us of
  // fabric traffic at 248 workgroups -- is paid back by the shorter k-loop
  // only on long K (A/B r05 ks2, us, 8-wave k-split tile vs K-split: 205
  // blocks of 4096^2 at K = 4096 40.2 vs 42.0 (S = 4), K = 8192 68.9 vs
  // 62.9 (S = 8); 60 blocks of 2048 x 4096, K = 4096 30.8 vs 31.0; 300
  // blocks, K = 2048 37.5 vs 38.0).
  if (p->num_rows > kMaxGroupRows || p->k_limit < Knob(kKnobSddKsplitMinK) ||
      p->k_limit % 128 != 0)
    return false;
  if (stream == hipStreamPerThread) return false;  // many streams, one handle
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const int cus = DeviceCUs(dev);
  if (cus <= 0) return false;
  // groups: sum over rows of ceil(n_r / 4) <= (blocks + 3 rows) / 4
  const long long blocks = p->num_tiles;
  const long long groups_ub = (blocks + 3LL * p->num_rows) / 4;
  if (groups_ub * 2 > cus) return false;
  const long long span = 32LL * p->d_ld + (long long)p->j_limit * 2;
  if (span > kMaxLaneOffset) return false;
  GemmParams q = *p;
  q.c_offsets = static_cast<const int *>(c.offsets);
  if (!Sdd4wApplies(q, true, ta, tb)) return false;
  std::lock_guard<std::mutex> lock(g_pairs_mu);
  PairSlot dry_slot;
  int capturing = 0;
  PairSlot *slot = AcquirePairSlot(stream, dry, &dry_slot, &capturing);
  if (slot == nullptr || cus > slot->slots) return false;
  *p = q;
  p->num_tiles = cus;
  p->pair = 1;  // (the epoch and capture protocol of pair launches)
  if (!dry) BindPairSlot(p, slot, capturing);
  p->pair_fault = Knob(kKnobPairFault);
  p->sdd_ksplit = max_s;
  return true;
}

// Tall sparse operands (more block-rows than the in-kernel row ranking
// handles, so no LPT order and no pair balancing) have many more tiles than
// CUs: they run on CfgTall, two workgroups per CU.
// dry: decide only (DsdPlan), no counter allocated.
bool UseTall(GemmParams *p, hipStream_t stream, bool dry = false) {
  // knob "tall": 0 never, 2 always (experiments), 1 (default): tall only.
  const int mode = Knob(kKnobTall);
  if (mode == 0) return false;
  if (mode == 2) {
    // Forced tall (experiments): drop every pair-launch setting PreparePairs
    // made, split mode's grid and tile width included.
    p->pair = 0;
    p->pair_split = 1;
    p->split_bn = 0;
    p->grid = 0;
  } else if (p->num_rows <= kLptRows || p->pair != 0) {
    return false;
  }
  p->num_jtiles = (p->j_limit + CfgTall::kBN - 1) / CfgTall::kBN;
  p->num_tiles = p->num_rows * p->num_jtiles;
  // Persistent: one workgroup per slot; the first `slots` tiles go by
  // workgroup index, the rest are fetched from a per-stream counter. Short
  // tiles (most rows of a tall 2% operand hold 0-2 blocks) otherwise leave
  // ~20% of the slots idle between a workgroup's end and the next dispatch
  // (r02 timeline: 400-460 of 512 resident); a static tile stride instead
  // loses more to imbalance (403 vs 337 us, config 5).
  const int persistent = Knob(kKnobTallPersistent);
  int dev = 0;
  const int cus = hipGetDevice(&dev) == hipSuccess ? DeviceCUs(dev) : 0;
  const int slots = cus * CfgTall::kWGs;
  if (!persistent || slots <= 0 || p->num_tiles <= slots) return true;
  if (stream == hipStreamPerThread) return true;  // many streams, one handle
  // A captured launch gets a counter pair of its own capture (the kernel
  // leaves it at zero, so every replay starts clean).
  unsigned long long capture = 0;
  const int capturing = CaptureState(stream, &capture);
  if (capturing < 0) return true;
  std::lock_guard<std::mutex> lock(g_pairs_mu);
  CounterSlot *table = capturing ? g_capture_counters : g_counters;
  const int n_table = capturing ? kMaxCaptureSlots : kMaxPairSlots;
  CounterSlot *slot = nullptr;
  for (int i = 0; i < n_table; ++i) {
    CounterSlot &c = table[i];
    if (c.counter != nullptr && c.device == dev && c.stream == stream &&
        c.capture == capture) {
      slot = &c;
      break;
    }
  }
  // (a released capture slot is re-tied as in PreparePairs: the kernel left
  // its counter pair at zero)
  if (slot == nullptr && capturing) {
    for (int i = 0; i < n_table; ++i) {
      CounterSlot &c = table[i];
      if (c.counter != nullptr && c.device == dev &&
          c.released.load(std::memory_order_acquire) != 0) {
        slot = &c;
        if (!dry) {
          c.stream = stream;
          c.capture = capture;
          c.released.store(0, std::memory_order_relaxed);
          (void)TieToCapturedGraph(stream, &c.released);
        }
        break;
      }
    }
  }
  if (slot == nullptr) {
    for (int i = 0; i < n_table; ++i)
      if (table[i].counter == nullptr) {
        slot = &table[i];
        break;
      }
    if (slot == nullptr) {
      if (!dry) WarnSlotsFull(capturing ? 3 : 1);
      return true;
    }
    if (dry) {  // the counter a launch would allocate
      p->grid = slots;
      p->persistent = 1;
      return true;
    }
    void *ctr = nullptr;
    if (AllocZeroed(&ctr, 2 * sizeof(unsigned long long), dev) != hipSuccess)
      return true;
    slot->device = dev;
    slot->stream = stream;
    slot->capture = capture;
    slot->counter = static_cast<unsigned long long *>(ctr);
    slot->released.store(0, std::memory_order_relaxed);
    if (capturing) (void)TieToCapturedGraph(stream, &slot->released);
  }
  p->grid = slots;
  p->persistent = 1;
  p->tile_counter = slot->counter;
  return true;
}

}  // namespace

// ---- shared entry points -------------------------------------------------

// Tall DSD NN on the 4-wave kernel, persistent (dsd4w.hip kEpi 7): one
// workgroup per CU walks a cost-balanced contiguous range of the
// panel-major block sequence (512-column panels) and stores each 128 x 512
// tile through a free ring slot as soon as its last block is done, the next
// tile's first DMAs in flight meanwhile; the empty rows' tiles are
// zero-filled after, an equal share per workgroup. Needs whole 512-column
// panels, at most 128 blocks and 64 zero chunks per workgroup, and rows that
// fit the LDS copy of the offsets.
static bool UseTallPipe(const GemmParams &p, long long blocks, long long row_max, bool ta,
                        bool tb) {
  if (Knob(kKnobTall4w) == 0 || !Dsd4wEnabled() || ta || tb) return false;
  if (p.pair != 0 || p.pair_split > 1 || CfgSparse::kBN != 512) return false;
  if (p.j_limit % 512 != 0 || p.num_rows > 32767 || blocks <= 0) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const int cus = DeviceCUs(dev);
  if (cus <= 0) return false;
  // blocks per workgroup: a weighted share (a tile weighs its blocks + 1:
  // blocks + non-empty rows per panel) plus the tile the cut runs into
  // (weight w quarter blocks per tile: blocks + w / 4 x non-empty rows)
  const long long fw = Knob(kKnobTallFlushW);
  const long long per =
      ((4 * blocks + fw * std::min<long long>(blocks, p.num_rows)) * (p.j_limit / 512) +
       4LL * cus - 1) / (4LL * cus);
  // (the empty rows' zero chunks: a share of at most panels x rows; the
  // odd-XCD share scales both by up to 2 max(odd, 100) / (100 + odd))
  const long long odd = Knob(kKnobTallOddShare), big = std::max<long long>(odd, 100);
  const long long zero_per =
      ((long long)(p.j_limit / 512) * p.num_rows * 2 * big + cus * (100 + odd) - 1) /
      (cus * (100 + odd));
  const long long per_x = (per * 2 * big + (100 + odd) - 1) / (100 + odd) + 1;
  return per_x + row_max <= 128 && zero_per <= 63 && blocks < (1LL << 24) &&
         p.j_limit / 512 < 256;
}

// ---- SDD with B stored transposed, over operands past the MALL -------------
// SDD NT / TT read B^T's rows 256 B per k-block. While A and B fit the
// 256-MB Infinity Cache (MALL) that costs nothing (NT 8192^3 runs at NN's
// speed), past it the misses go to HBM: SDD NT 16384^3 at 50% ran 5231 us
// against NN's 3516. There, B is transposed
// once into a library-owned buffer ([K][N], layout.hip, ~2 K N 2 bytes of
// HBM traffic) and the N-major kernel (NN / TN) runs on it. Gate: B's
// K N 2 bytes >= knob sdd_bt_min_mib MiB, and the product's FLOPs per byte
// of B (blocks 128^2 2 K / (K N 2) = 16384 blocks / N) >= kBtMinRatio, so
// the copy is a small part of the launch (16384^3: 50% 8192, dense 16384,
// 10% 1639 -- below; MegaBlocks' x.w1^T 1024 -- below); the N-major path
// must be the 4-wave grouped kernel. Eager launches only: a stream being
// captured keeps the NT / TT kernel (the buffer is allocated on first use).
// One buffer per (device, stream), grown as needed, kept for the process
// (INTEGRATION.md 3b); stream order makes it safe to reuse.
constexpr long long kBtMinRatio = 3000;
struct BtSlot {
  int device = -1;
  hipStream_t stream = nullptr;
  void *data = nullptr;
  size_t bytes = 0;
};
static BtSlot g_bt[kMaxPairSlots];
// Held from choosing the buffer until the transpose and the product are
// enqueued, so another thread cannot grow (free) the buffer of the same
// stream in between; taken before g_pairs_mu, never while holding it.
static std::mutex g_bt_mu;

static bool UseBtTranspose(const Matrix &a, bool ta, const Matrix &b, bool tb,
                           const BlockMatrix &c, hipStream_t stream) {
  if (!tb || stream == hipStreamPerThread) return false;  // (many streams, one handle)
  const long long min_mib = Knob(kKnobSddBtMinMib);
  if (min_mib <= 0) return false;
  const long long n = b.rows, k = b.cols;  // B^T stored [N][K]
  // (layout.hip moves 16-byte vectors: a 16-byte aligned B)
  if (n % 64 != 0 || k % 64 != 0 || n * k * 2 < (min_mib << 20) ||
      (reinterpret_cast<uintptr_t>(b.data) & 15) != 0)
    return false;
  const long long blocks = c.nonzeros / (kBlock * kBlock);
  if (blocks * 16384 < kBtMinRatio * n) return false;
  unsigned long long id = 0;
  if (CaptureState(stream, &id) != 0) return false;
  GemmParams p;
  const Matrix bt((int)k, (int)n, b.data);
  return PrepareSdd(a, ta, bt, false, c, &p) == Status::kOk && UseGroupedSdd(&p, c, false) &&
         Dsd4wEnabled() && Sdd4wApplies(p, true, ta, false, blocks);
}

// The same for DSD NT over a nearly dense A (out = A . B with B^T stored
// [N][K] past the MALL): the sweep's DSD NT 16384^3 dense ran 7620 us
// against NN's 6354, while at 50% NT is as fast as NN (3352 vs 3397 us), so
// the gate asks for >= kDsdBtMinRatio FLOPs per byte of B, 16384 blocks / K
// (16384^3: dense 16384, 50% 8192).
constexpr long long kDsdBtMinRatio = 15000;
static bool UseBtTransposeDsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                              hipStream_t stream) {
  if (!tb || ta || stream == hipStreamPerThread) return false;
  const long long min_mib = Knob(kKnobSddBtMinMib);
  if (min_mib <= 0) return false;
  const long long n = b.rows, k = b.cols;  // B^T stored [N][K]
  // (layout.hip moves 16-byte vectors: a 16-byte aligned B)
  if (n % 64 != 0 || k % 64 != 0 || n * k * 2 < (min_mib << 20) ||
      (reinterpret_cast<uintptr_t>(b.data) & 15) != 0)
    return false;
  const long long blocks = a.nonzeros / (kBlock * kBlock);
  if (blocks * 16384 < kDsdBtMinRatio * k) return false;
  unsigned long long id = 0;
  return CaptureState(stream, &id) == 0;
}

// The transposed-B buffer of (device, stream), at least `bytes` (nullptr:
// none -- the table is full or the allocation failed; the caller keeps the
// NT / TT kernel). Caller holds g_bt_mu.
static void *BtBuffer(hipStream_t stream, size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  BtSlot *slot = nullptr;
  for (BtSlot &s : g_bt)
    if (s.data != nullptr && s.device == dev && s.stream == stream) slot = &s;
  if (slot == nullptr)
    for (BtSlot &s : g_bt)
      if (s.data == nullptr) {
        slot = &s;
        break;
      }
  if (slot == nullptr) return nullptr;
  if (slot->bytes < bytes) {
    if (slot->data != nullptr) {
      // the stream's earlier launches may still read the old buffer
      if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
      FreeQuiet(slot->data);
      slot->data = nullptr;
      slot->bytes = 0;
    }
    if (hipMalloc(&slot->data, bytes) != hipSuccess) {
      slot->data = nullptr;
      return nullptr;
    }
    slot->bytes = bytes;
    slot->device = dev;
    slot->stream = stream;
  }
  return slot->data;
}

hipError_t RunDsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const Matrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *st_out) {
  GemmParams p;
  bool needs_meta = false;
  const Status st = PrepareDsd(a, ta, b, tb, c, &p, &needs_meta);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (UseBtTransposeDsd(a, ta, b, tb, stream)) {
    std::lock_guard<std::mutex> lock(g_bt_mu);
    void *bt = BtBuffer(stream, (size_t)b.rows * b.cols * 2);
    if (bt != nullptr) {
      const hipError_t e = LaunchTranspose16(b.data, b.rows, b.cols, bt, stream);
      if (e != hipSuccess) return e;
      return RunDsd(a, ta, Matrix(b.cols, b.rows, bt), false, c, dtype, build_meta, stream,
                    st_out);
    }
  }
  if (needs_meta && build_meta) {
    const hipError_t e = BuildTransposed(a, stream);
    if (e != hipSuccess) return e;
  }
  p.debug = g_debug;
  p.xcd_rows = Knob(kKnobXcdRows);
  PreparePairs(&p, a.nonzeros / (kBlock * kBlock), stream);
  const GemmParams p0 = p;  // (before the tall configuration)
  // decide without allocating first: the tall pipeline needs no persistent
  // tile counter, so only the 8-wave tall path takes one
  GemmParams pd = p;
  const bool tall = UseTall(&pd, stream, /*dry=*/true);
  if (tall && UseTallPipe(p0, a.nonzeros / (kBlock * kBlock),
                          ((long long)a.cols + kBlock - 1) / kBlock, ta, tb)) {
    GemmParams q = p0;
    q.persistent = 0;
    q.num_jtiles = q.j_limit / 512;
    q.tall_flush_w = Knob(kKnobTallFlushW);
    q.tall_odd_share = Knob(kKnobTallOddShare);
    int dev = 0;
    q.num_tiles = hipGetDevice(&dev) == hipSuccess ? DeviceCUs(dev) : 0;
    return LaunchDsd4w(dtype, q, 7, false, stream, false, false);
  }
  if (tall) (void)UseTall(&p, stream);
  if (Dsd4wEnabled() &&
      Dsd4wApplies(p, Dsd4wForced() ? (1LL << 40) : a.nonzeros / (kBlock * kBlock),
                   !ta, tb, false, tall)) {
    // Default epilogue by density: below a mean of 12 blocks per block-row
    // the copy-out interleaved with the staging (kEpi 5) is ahead (DSD NN
    // 4096^3 A/B r04ae, two runs: 10% +1.5 / +1.2%, 30% +1.0 / +0.5%), at
    // 50% behind (-0.6 / -0.3%).
    int epi = Dsd4wEpi();
    if (Dsd4wMode() == 1 && a.nonzeros / (kBlock * kBlock) < 12LL * p.num_rows)
      epi = 5;
    return LaunchDsd4w(dtype, p, epi, tb && !ta, stream, ta && !tb, ta && tb);
  }
  return LaunchBlockGemm(dtype, false, !ta, tb, false, tall, p, stream);
}

hipError_t RunDds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const Matrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *st_out) {
  GemmParams p;
  bool needs_meta = false;
  const Status st = PrepareDds(a, ta, b, tb, c, &p, &needs_meta);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (needs_meta && build_meta) {
    const hipError_t e = BuildTransposed(b, stream);
    if (e != hipSuccess) return e;
  }
  p.debug = g_debug;
  p.xcd_rows = Knob(kKnobXcdRows);
  PreparePairs(&p, b.nonzeros / (kBlock * kBlock), stream);
  const bool tall = UseTall(&p, stream);
  if (Dsd4wEnabled() &&
      Dds4wApplies(p, Dsd4wForced() ? (1LL << 40) : b.nonzeros / (kBlock * kBlock),
                   tb, !ta, true, tall)) {
    // (the two-panel pair placement, heavy pairs on the odd XCDs: DDS NN
    // A/B r05 dx, same process, mode 0 -> 3: 10% 24.49 -> 24.41, 20% 32.44
    // -> 32.33, 30% 40.03 -> 38.69, 50% 56.75 -> 55.06, 90% 89.76 -> 87.64 us)
    if (p.pair_xcd2 != 0) p.pair_xcd2 = Knob(kKnobDdsXcd2);
    return LaunchDds4w(dtype, p, Dsd4wEpi(), tb && !ta, stream, ta && !tb, ta && tb);
  }
  return LaunchBlockGemm(dtype, false, /*s_kc=*/tb, /*d_kc=*/!ta,
                         /*out_t=*/true, tall, p, stream);
}

hipError_t RunSdd(const Matrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, int dtype, hipStream_t stream,
                  Status *st_out) {
  GemmParams p;
  const Status st = PrepareSdd(a, ta, b, tb, c, &p);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (UseBtTranspose(a, ta, b, tb, c, stream)) {
    std::lock_guard<std::mutex> lock(g_bt_mu);
    void *bt = BtBuffer(stream, (size_t)b.rows * b.cols * 2);
    if (bt != nullptr) {
      const hipError_t e = LaunchTranspose16(b.data, b.rows, b.cols, bt, stream);
      if (e != hipSuccess) return e;
      return RunSdd(a, ta, Matrix(b.cols, b.rows, bt), false, c, dtype, stream, st_out);
    }
  }
  p.debug = g_debug;
  const int blocks = p.num_tiles;
  const bool grouped = UseGroupedSdd(&p, c, tb);
  if (!grouped && PrepareSddKsplit(&p, c, ta, tb, stream))
    return LaunchSdd4w(dtype, p, ta, tb, Dsd4wEpi(), stream);
  if (Dsd4wEnabled() && Sdd4wApplies(p, grouped, ta, tb, c.nonzeros / (kBlock * kBlock))) {
    p.sdd_order = Knob(kKnobSddOrder);
    p.sdd_krot = Knob(kKnobSddKrot);
    const int spread = Knob(kKnobSddSpread);
    p.sdd_spread = spread == 1 || (spread == 2 && tb && !ta) ? 1 : 0;
    // Tail split (block_gemm.h sdd_tail_rows): with K >= sdd_tail_min_k a
    // grouped round is long, so the rows past the full rounds are better
    // served one block per workgroup by the 8-wave k-split tile, launched
    // right behind on the same stream (both launches find the same R0).
    // Only while A and B fit the 256-MB MALL: that tile streams a whole
    // row panel of A and column panel of B per block, and past the MALL it
    // ran slower than the round it saves (SDD 16384^3 50%: NN 3428 -> 3644
    // us, 8192^3 50%: 494 -> 445 us, profiles/r06/ab/sdd_tail_ab.jsonl).
    int dev = 0;
    const long long tail_k = Knob(kKnobSddTailMinK);
    const long long ab_bytes = 2LL * p.k_limit * ((long long)p.num_rows * kBM + p.j_limit);
    const bool tail = tail_k > 0 && p.k_limit >= tail_k && ab_bytes <= (256LL << 20) &&
                      hipGetDevice(&dev) == hipSuccess && DeviceCUs(dev) > 0;
    if (tail) {
      p.sdd_tail = 1;
      p.tail_cus = DeviceCUs(dev);
    }
    const hipError_t e = LaunchSdd4w(dtype, p, ta, tb, Dsd4wEpi(), stream);
    if (e != hipSuccess || !tail) return e;
    GemmParams q = p;
    q.num_tiles = blocks;
    q.grid = p.tail_cus;
    q.sdd_order = 0;
    return LaunchBlockGemm(dtype, true, /*s_kc=*/!ta, /*d_kc=*/tb, false,
                           /*grouped=*/false, q, stream);
  }
  return LaunchBlockGemm(dtype, true, /*s_kc=*/!ta, /*d_kc=*/tb, false,
                         grouped, p, stream);
}

hipError_t RunSsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *st_out) {
  GemmParams p;
  bool needs_meta = false;
  const Status st = PrepareSsd(a, ta, b, tb, c, &p, &needs_meta);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (needs_meta && build_meta) {
    const hipError_t e = BuildTransposed(a, stream);
    if (e != hipSuccess) return e;
  }
  p.debug = g_debug;
  return LaunchBlockGemmSparseIn(dtype, /*s_kc=*/!ta, /*d_kc=*/tb,
                                 /*out_t=*/false, p, stream);
}

hipError_t RunSds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const BlockMatrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *st_out) {
  GemmParams p;
  bool needs_meta = false;
  const Status st = PrepareSds(a, ta, b, tb, c, &p, &needs_meta);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (needs_meta && build_meta) {
    const hipError_t e = BuildTransposed(b, stream);
    if (e != hipSuccess) return e;
  }
  p.debug = g_debug;
  return LaunchBlockGemmSparseIn(dtype, /*s_kc=*/tb, /*d_kc=*/!ta,
                                 /*out_t=*/true, p, stream);
}

hipError_t RunDss(const BlockMatrix &a, bool ta, const BlockMatrix &b,
                  bool tb, const Matrix &c, int dtype, bool build_meta_a,
                  bool build_meta_b, hipStream_t stream, Status *st_out) {
  GemmParams p;
  bool meta_a = false, meta_b = false;
  const Status st = PrepareDss(a, ta, b, tb, c, &p, &meta_a, &meta_b);
  *st_out = st;
  if (st != Status::kOk) return hipSuccess;
  if (meta_a && build_meta_a) {
    const hipError_t e = BuildTransposed(a, stream);
    if (e != hipSuccess) return e;
  }
  if (meta_b && build_meta_b) {
    const hipError_t e = BuildTransposed(b, stream);
    if (e != hipSuccess) return e;
  }
  p.debug = g_debug;
  return LaunchBlockGemmDss(dtype, /*s_kc=*/!ta, /*d_kc=*/tb, p, stream);
}

}  // namespace sputnik_amd

// ---- C++ API (drop-in for the reference's sputnik::block) ---------------

namespace sputnik {
namespace block {

using sputnik_amd::Status;

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e =
      sputnik_amd::RunDsd(a, transpose_a, b, transpose_b, c, (int)dtype,
                          a.create_metadata, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "dsd");
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream) {
  BlockMatrix acp = a;
  acp.create_metadata = false;
  return Matmul(acp, transpose_a, b, transpose_b, c, dtype, stream);
}

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, Matrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, Matrix c, hipStream_t stream) {
  return MatmulEx(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e =
      sputnik_amd::RunDds(a, transpose_a, b, transpose_b, c, (int)dtype,
                          b.create_metadata, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "dds");
}

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream) {
  BlockMatrix bcp = b;
  bcp.create_metadata = false;
  return Matmul(a, transpose_a, bcp, transpose_b, c, dtype, stream);
}

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, hipStream_t stream) {
  return MatmulEx(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t Matmul(const Matrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e = sputnik_amd::RunSdd(a, transpose_a, b, transpose_b, c,
                                           (int)dtype, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "sdd");
}

hipError_t Matmul(const Matrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

// SSD (reference sputnik/block/ssd/ssd.h:10-22) and SDS (sds.h:10-22).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e =
      sputnik_amd::RunSsd(a, transpose_a, b, transpose_b, c, (int)dtype,
                          a.create_metadata, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "ssd");
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, BlockMatrix c, DataType dtype,
                    hipStream_t stream) {
  BlockMatrix acp = a;
  acp.create_metadata = false;
  return Matmul(acp, transpose_a, b, transpose_b, c, dtype, stream);
}

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, BlockMatrix c, hipStream_t stream) {
  return MatmulEx(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e =
      sputnik_amd::RunSds(a, transpose_a, b, transpose_b, c, (int)dtype,
                          b.create_metadata, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "sds");
}

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, BlockMatrix c, DataType dtype,
                    hipStream_t stream) {
  BlockMatrix bcp = b;
  bcp.create_metadata = false;
  return Matmul(a, transpose_a, bcp, transpose_b, c, dtype, stream);
}

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, BlockMatrix c, hipStream_t stream) {
  return MatmulEx(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

// DSS (reference sputnik/block/dss/dss.h:10-22).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream) {
  Status st;
  const hipError_t e = sputnik_amd::RunDss(
      a, transpose_a, b, transpose_b, c, (int)dtype, a.create_metadata,
      b.create_metadata, stream, &st);
  return st == Status::kOk ? e : sputnik_amd::OrAbort(st, "dss");
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream) {
  BlockMatrix acp = a, bcp = b;
  acp.create_metadata = false;
  bcp.create_metadata = false;
  return Matmul(acp, transpose_a, bcp, transpose_b, c, dtype, stream);
}

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, hipStream_t stream) {
  return Matmul(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, hipStream_t stream) {
  return MatmulEx(a, transpose_a, b, transpose_b, c, DataType::kF16, stream);
}

hipError_t RowIndices(BlockMatrix a, short *row_indices, hipStream_t stream) {
  if (AsInt(a.block_size) == 0) return hipErrorNotSupported;
  return sputnik_amd::LaunchRowIndices(a.rows / AsInt(a.block_size),
                                       static_cast<const int *>(a.offsets),
                                       row_indices, stream);
}

hipError_t Bitmask(BlockMatrix m, hipStream_t stream) {
  // bitmask.cu:8-16: the orientation follows offsets_t.
  const bool trans = m.offsets_t != nullptr;
  const int b = AsInt(m.block_size);
  if (b == 0) return hipErrorNotSupported;
  SPUTNIK_CHECK(m.bitmask);
  const int block_rows = (trans ? m.cols : m.rows) / b;
  const int block_cols = (trans ? m.rows : m.cols) / b;
  return sputnik_amd::LaunchBitmask(
      block_rows, block_cols,
      static_cast<const int *>(trans ? m.offsets_t : m.offsets),
      static_cast<const short *>(trans ? m.indices_t : m.indices),
      static_cast<unsigned long long *>(m.bitmask), stream);
}

hipError_t Transpose(BlockMatrix a, hipStream_t stream) {
  // transpose.cu:107-109 checks the three workspaces; with no nonzero block
  // the two per-block ones are legitimately empty.
  SPUTNIK_CHECK(a.offsets_t);
  if (a.nonzeros > 0) {
    SPUTNIK_CHECK(a.indices_t);
    SPUTNIK_CHECK(a.block_offsets);
  }
  return sputnik_amd::BuildTransposed(a, stream);
}

}  // namespace block
}  // namespace sputnik

namespace sputnik_amd {

int StatusCode(Status st) { return AsCode(st); }

int SddPlan(const void *a, bool ta, const void *b, bool tb, const void *c) {
  if (!a || !b || !c) return -1;
  GemmParams p;
  const BlockMatrix &cm = *static_cast<const BlockMatrix *>(c);
  if (PrepareSdd(*static_cast<const Matrix *>(a), ta,
                 *static_cast<const Matrix *>(b), tb, cm, &p) != Status::kOk)
    return -1;
  if (UseGroupedSdd(&p, cm, tb)) return 1;
  return PrepareSddKsplit(&p, cm, ta, tb, nullptr, /*dry=*/true) ? 2 : 0;
}

// The kernel behind SddPlan's tile plan (what RunSdd launches): 0 the
// 8-wave k-split 128 x 128 block tile, 1 grouped tiles on the 8-wave
// kernel, 2 the 4-wave K-split, 3 grouped tiles on the 4-wave kernel, -1
// rejected.
int SddKernel(const void *a, bool ta, const void *b, bool tb, const void *c) {
  const int plan = SddPlan(a, ta, b, tb, c);
  if (plan != 1) return plan;
  GemmParams p;
  const BlockMatrix &cm = *static_cast<const BlockMatrix *>(c);
  if (UseBtTranspose(*static_cast<const Matrix *>(a), ta, *static_cast<const Matrix *>(b),
                     tb, cm, nullptr))
    return 4;
  if (PrepareSdd(*static_cast<const Matrix *>(a), ta,
                 *static_cast<const Matrix *>(b), tb, cm, &p) != Status::kOk ||
      !UseGroupedSdd(&p, cm, tb))
    return -1;
  return Dsd4wEnabled() && Sdd4wApplies(p, true, ta, tb, cm.nonzeros / (kBlock * kBlock))
             ? 3
             : 1;
}

// Which kernel RunDds would launch on `stream` (no launch, nothing
// allocated): 0 the 8-wave 128 x 512 tile, 1 the 4-wave kernel, 2 the tall
// configuration, 3 split mode on the 8-wave kernel, -1 rejected.
int DdsPlan(const void *a, bool ta, const void *b, bool tb, const void *c,
            hipStream_t stream) {
  if (!a || !b || !c) return -1;
  GemmParams p;
  bool needs_meta = false;
  const BlockMatrix &bm = *static_cast<const BlockMatrix *>(b);
  if (PrepareDds(*static_cast<const Matrix *>(a), ta, bm, tb,
                 *static_cast<const Matrix *>(c), &p, &needs_meta) != Status::kOk)
    return -1;
  PreparePairs(&p, bm.nonzeros / (kBlock * kBlock), stream, /*dry=*/true);
  const bool tall = UseTall(&p, stream, /*dry=*/true);
  if (Dsd4wEnabled() &&
      Dds4wApplies(p, Dsd4wForced() ? (1LL << 40) : bm.nonzeros / (kBlock * kBlock), tb,
                   !ta, true, tall))
    return 1;
  if (tall) return 2;
  if (p.pair != 0 && p.pair_split > 1) return 3;
  return 0;
}

// Which kernel RunDsd would launch for this problem on `stream` (no
// launch): 0 the 8-wave 128 x 512 tile, 1 the 4-wave hand-scheduled kernel
// (dsd4w.hip), 2 the tall configuration, 3 split mode, 4 the tall
// pipeline (4-wave, persistent), -1 rejected. Read-only:
// it makes the workspace decisions a launch would make without allocating,
// re-tying or advancing any workspace (safe during a capture). (DSD NT
// that transposes B first, UseBtTransposeDsd: the plan of the NN product
// that follows.)
int DsdPlan(const void *a, bool ta, const void *b, bool tb, const void *c,
            hipStream_t stream) {
  if (!a || !b || !c) return -1;
  GemmParams p;
  bool needs_meta = false;
  const BlockMatrix &am = *static_cast<const BlockMatrix *>(a);
  const Matrix &bm = *static_cast<const Matrix *>(b);
  if (UseBtTransposeDsd(am, ta, bm, tb, stream)) {
    const Matrix bt(bm.cols, bm.rows, bm.data);
    if (PrepareDsd(am, ta, bm, tb, *static_cast<const Matrix *>(c), &p, &needs_meta) ==
        Status::kOk)
      return DsdPlan(a, ta, &bt, false, c, stream);
  }
  if (PrepareDsd(am, ta, *static_cast<const Matrix *>(b), tb,
                 *static_cast<const Matrix *>(c), &p, &needs_meta) != Status::kOk)
    return -1;
  PreparePairs(&p, am.nonzeros / (kBlock * kBlock), stream, /*dry=*/true);
  const GemmParams p0 = p;
  const bool tall = UseTall(&p, stream, /*dry=*/true);
  if (tall && UseTallPipe(p0, am.nonzeros / (kBlock * kBlock),
                          ((long long)am.cols + kBlock - 1) / kBlock, ta, tb))
    return 4;
  if (Dsd4wEnabled() &&
      Dsd4wApplies(p, Dsd4wForced() ? (1LL << 40) : am.nonzeros / (kBlock * kBlock),
                   !ta, tb, false, tall))
    return 1;
  if (tall) return 2;
  if (p.pair != 0 && p.pair_split > 1) return 3;
  return 0;
}

// Host-only acceptance test (no launch, no device needed): op 0 = DSD
// (a: block, b/c: dense), 1 = DDS (b: block), 2 = SDD (c: block), 3 = SSD
// (a, c: block), 4 = SDS (b, c: block), 5 = DSS (a, b: block). The C
// descriptors share the C++ layout (static_asserts in c_api.cpp).
bool CanImplement(int op, const void *a, bool ta, const void *b, bool tb,
                  const void *c) {
  if (!a || !b || !c) return false;
  GemmParams p;
  bool meta = false;
  Status st = Status::kNoKernel;
  if (op == 0) {
    st = PrepareDsd(*static_cast<const BlockMatrix *>(a), ta,
                    *static_cast<const Matrix *>(b), tb,
                    *static_cast<const Matrix *>(c), &p, &meta);
  } else if (op == 1) {
    st = PrepareDds(*static_cast<const Matrix *>(a), ta,
                    *static_cast<const BlockMatrix *>(b), tb,
                    *static_cast<const Matrix *>(c), &p, &meta);
  } else if (op == 2) {
    st = PrepareSdd(*static_cast<const Matrix *>(a), ta,
                    *static_cast<const Matrix *>(b), tb,
                    *static_cast<const BlockMatrix *>(c), &p);
  } else if (op == 3) {
    st = PrepareSsd(*static_cast<const BlockMatrix *>(a), ta,
                    *static_cast<const Matrix *>(b), tb,
                    *static_cast<const BlockMatrix *>(c), &p, &meta);
  } else if (op == 4) {
    st = PrepareSds(*static_cast<const Matrix *>(a), ta,
                    *static_cast<const BlockMatrix *>(b), tb,
                    *static_cast<const BlockMatrix *>(c), &p, &meta);
  } else if (op == 5) {
    bool meta_b = false;
    st = PrepareDss(*static_cast<const BlockMatrix *>(a), ta,
                    *static_cast<const BlockMatrix *>(b), tb,
                    *static_cast<const Matrix *>(c), &p, &meta, &meta_b);
  }
  return st == Status::kOk;
}

}  // namespace sputnik_amd

// Experiment hook (not part of include/sputnik_amd.h): per-segment cycle
// sums / timelines of SPUTNIK_EXP & 128 / 512 builds (scripts/exp_build.sh).
// Only experiment builds export it; the shipped library has no such entry.
#if SPUTNIK_EXP != 0
extern "C" void sputnik_exp_set_debug(void *buffer) {
  sputnik_amd::g_debug = static_cast<unsigned long long *>(buffer);
}
#endif
