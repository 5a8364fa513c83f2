/*
 * mxp_batch.h -- host-side columnar attribute-bag batch (the input format of the C-ABI).
 *
 * A batch is N request attribute bags laid out column-wise, one column per attribute name, so the
 * engine can pack exactly the columns a rule set references into its device SoA buffers.  It is the
 * batched stand-in for `attribute.Bag` (mixer/pkg/attribute/bag.go:18-31): `Get(name)` on request r
 * returns (kinds[c][r], values[c][r]) of the column whose name is `name`, or "not found" when the
 * column is absent from the batch or kinds[c][r] == MXP_ABSENT.
 *
 * Each value carries the Go dynamic type it had in the bag (the interpreter type-asserts at
 * runtime, mixer/pkg/il/interpreter/interpreterRun.go:455-708), encoded by `mxp_kind`:
 *   STRING     values = batch string id (index into the string table below)
 *   INT64      values = the int64 bits
 *   DOUBLE     values = math.Float64bits
 *   BOOL       values = 0 / 1
 *   DURATION   values = int64 nanoseconds (time.Duration)
 *   TIMESTAMP  values = index into time_sec/time_nsec (time.Time, compared as instants)
 *   BYTES      values = batch string id of the raw bytes ([]byte, e.g. net.IP)
 *   STRING_MAP values = map id: entries [map_offsets[id], map_offsets[id+1]) of (key, value) string
 *                       ids, keys unique within a map
 *   OTHER      values = batch string id of the value's Go `%v` text (any other Go type, e.g. `int`)
 *
 * Strings are byte strings: string id s spans str_bytes[str_offsets[s] .. str_offsets[s+1]).
 * The same bytes may appear under several ids; the engine compares bytes, never batch ids.
 */
#ifndef MXP_BATCH_H
#define MXP_BATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mxp_kind {
    MXP_ABSENT = 0,
    MXP_STRING = 1,
    MXP_INT64 = 2,
    MXP_DOUBLE = 3,
    MXP_BOOL = 4,
    MXP_DURATION = 5,
    MXP_TIMESTAMP = 6,
    MXP_BYTES = 7,
    MXP_STRING_MAP = 8,
    MXP_OTHER = 9
};

typedef struct mxp_bag_batch {
    uint32_t n_requests;
    uint32_t n_columns;
    const char* const* column_names;   /* [n_columns] NUL-terminated attribute names        */
    const uint8_t* const* kinds;       /* [n_columns] -> uint8_t[n_requests]  (mxp_kind)    */
    const uint64_t* const* values;     /* [n_columns] -> uint64_t[n_requests]               */

    uint32_t n_strings;
    const uint8_t* str_bytes;
    const uint64_t* str_offsets;       /* [n_strings + 1]                                    */

    uint32_t n_times;
    const int64_t* time_sec;           /* [n_times] Unix seconds                             */
    const int32_t* time_nsec;          /* [n_times] nanoseconds in [0, 1e9)                  */

    uint32_t n_maps;
    const uint64_t* map_offsets;       /* [n_maps + 1]                                       */
    const uint32_t* map_keys;          /* [map_offsets[n_maps]] string ids                   */
    const uint32_t* map_values;        /* [map_offsets[n_maps]] string ids                   */
} mxp_bag_batch;

#ifdef __cplusplus
}
#endif

#endif /* MXP_BATCH_H */
