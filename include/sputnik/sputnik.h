// sputnik-amd umbrella header. Replaces reference sputnik/sputnik.h:18-25 for
// the block-sparse hot path (DSD, DDS, SDD, RowIndices). SSD/SDS/DSS are out of
// scope and are not declared.
#ifndef SPUTNIK_SPUTNIK_H_
#define SPUTNIK_SPUTNIK_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dsd/dsd.h"
#include "sputnik/block/dds/dds.h"
#include "sputnik/block/sdd/sdd.h"
#include "sputnik/block/row_indices/row_indices.h"
#include "sputnik/block/transpose/transpose.h"

#endif  // SPUTNIK_SPUTNIK_H_
