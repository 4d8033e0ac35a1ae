// sputnik-amd: host entry points shared by the C++ API and the C-ABI.
#ifndef SPUTNIK_AMD_API_INTERNAL_H_
#define SPUTNIK_AMD_API_INTERNAL_H_

#include "sputnik/block/arguments.h"

namespace sputnik_amd {

// Outcome of the host-side acceptance checks of one call.
enum class Status {
  kOk,
  kNotSupported,     // block size != 128 -> hipErrorNotSupported (dsd.cu:16)
  kNoKernel,         // reference: "No compatible kernel" -> abort
  kMissingMetadata,  // reference: SPUTNIK_CHECK(offsets_t ...) -> abort
  kMissingRowIndices,
};

using sputnik::block::BlockMatrix;
using sputnik::block::Matrix;

// Validate, optionally build transposed metadata, launch. A non-kOk *status
// means nothing was launched.
hipError_t RunDsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const Matrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *status);
hipError_t RunDds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const Matrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *status);
hipError_t RunSdd(const Matrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, int dtype, hipStream_t stream,
                  Status *status);

hipError_t RunSsd(const BlockMatrix &a, bool ta, const Matrix &b, bool tb,
                  const BlockMatrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *status);
hipError_t RunSds(const Matrix &a, bool ta, const BlockMatrix &b, bool tb,
                  const BlockMatrix &c, int dtype, bool build_meta,
                  hipStream_t stream, Status *status);

hipError_t RunDss(const BlockMatrix &a, bool ta, const BlockMatrix &b,
                  bool tb, const Matrix &c, int dtype, bool build_meta_a,
                  bool build_meta_b, hipStream_t stream, Status *status);

// hipError_t value the C-ABI returns for a status (never aborts).
int StatusCode(Status st);

// Host-only acceptance test. op 0 = DSD, 1 = DDS, 2 = SDD, 3 = SSD, 4 = SDS, 5 = DSS.
bool CanImplement(int op, const void *a, bool ta, const void *b, bool tb,
                  const void *c);

// SDD tile plan of a valid problem: 1 = grouped 128x512 tiles, 0 = one
// k-split 128x128 block per workgroup, -1 = rejected. Reads the CU count of
// the current device (no launch).
int SddPlan(const void *a, bool ta, const void *b, bool tb, const void *c);
// SDD kernel (dispatch.cpp SddKernel): 0 8-wave k-split tile, 1 8-wave
// grouped, 2 4-wave K-split, 3 4-wave grouped, -1 rejected.
int SddKernel(const void *a, bool ta, const void *b, bool tb, const void *c);
// DDS kernel plan (dispatch.cpp DdsPlan): 0 8-wave tile, 1 4-wave kernel,
// 2 tall, 3 split (8-wave), -1 rejected.
int DdsPlan(const void *a, bool ta, const void *b, bool tb, const void *c,
            hipStream_t stream);
// DSD kernel plan (dispatch.cpp DsdPlan): 0 8-wave tile, 1 4-wave kernel,
// 2 tall, 3 split mode, 4 tall pipeline, -1 rejected.
int DsdPlan(const void *a, bool ta, const void *b, bool tb, const void *c,
            hipStream_t stream);

// Pair hand-offs that timed out (see dispatch.cpp), and the test knob that
// makes every pair producer skip its publish.
int PairErrors();
void SetPairFault(int on);
int CaptureWorkspaces();
// DSD / DDS / grouped SDD: 4-wave kernel on (1) / off (0) / forced
// regardless of density with kEpi = mode - 2 (modes 2-7, dsd4w.h
// LaunchDsd4w); -1 queries. Returns the previous. (= knob "dsd4w")
int SelectDsdKernel(int four_wave);
bool Dsd4wEnabled();
bool Dsd4wForced();
int Dsd4wEpi();

// Unsupported tuning knobs (dispatch.cpp kKnobs: name, environment
// variable, default, range). Knob() reads one; TuningGet / TuningSet back
// sputnik_tuning_get / sputnik_tuning_set (INT_MIN: unknown name or value
// out of range).
enum KnobId {
  kKnobPairs,
  kKnobPairXcd2,
  kKnobSplit,
  kKnobSplitMinBn,
  kKnobDsd4w,
  kKnobGroupedSdd,
  kKnobGroupedMinPerCu,
  kKnobTall,
  kKnobTallPersistent,
  kKnobDdsXcd2,
  kKnobSdd4wMaxLd,
  kKnobPairFault,
  kKnobSddKsplit,
  kKnobSddKsplitMinK,
  kKnobSddOrder,
  kKnobTall4w,
  kKnobTallFlushW,
  kKnobTallOddShare,
  kKnobMinHandoff,
  kKnobXcdRows,
  kKnobSddKrot,
  kKnobSddSpread,
  kKnobSddBtMinMib,
  kKnobSddTailMinK,
  kNumKnobs
};
int Knob(KnobId k);
int TuningGet(const char *name);
int TuningSet(const char *name, int value);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_API_INTERNAL_H_
