// sputnik-amd umbrella header. Replaces reference sputnik/sputnik.h:18-25 for
// the six block-sparse products (DSD, DDS, SDD, SSD, SDS, DSS) and the
// metadata builders (RowIndices, Transpose, Bitmask).
#ifndef SPUTNIK_SPUTNIK_H_
#define SPUTNIK_SPUTNIK_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/bitmask/bitmask.h"
#include "sputnik/block/dsd/dsd.h"
#include "sputnik/block/dds/dds.h"
#include "sputnik/block/sdd/sdd.h"
#include "sputnik/block/ssd/ssd.h"
#include "sputnik/block/sds/sds.h"
#include "sputnik/block/dss/dss.h"
#include "sputnik/block/row_indices/row_indices.h"
#include "sputnik/block/transpose/transpose.h"

#endif  // SPUTNIK_SPUTNIK_H_
