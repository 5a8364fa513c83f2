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

/*
 * The narrow form of a batch (round 6): what crosses the host link is about a third smaller.  A
 * column whose kinds are all id kinds (STRING, BYTES, OTHER, TIMESTAMP, STRING_MAP) or BOOL / ABSENT
 * -- narrow[c] = 1 -- carries u32 values in values32[c]; any other column keeps its u64 values in
 * base.values[c].  String and map offsets are u32 (a batch's string bytes and map entries stay below
 * 4 GiB).  base.str_offsets and base.map_offsets are unused (NULL); everything else is base's.  The
 * engine widens on the device after the copies (mxp_batch_upload2).  A Go packer writes the ids
 * straight into u32 columns: the dictionary-encoded ids of the wire are 32-bit already
 * (dictState.go:75-82).
 */
typedef struct mxp_bag_batch2 {
    mxp_bag_batch base;
    const uint8_t* narrow;             /* [n_columns] 1: values32[c], 0: base.values[c]          */
    const uint32_t* const* values32;   /* [n_columns] -> uint32_t[n_requests] (narrow columns)   */
    const uint32_t* str_offsets32;     /* [n_strings + 1]                                        */
    const uint32_t* map_offsets32;     /* [n_maps + 1]                                           */
} mxp_bag_batch2;

/*
 * The wire form: N `CompressedAttributes` messages (istio.io/api mixer/v1 attributes.proto, the
 * Attributes of a CheckRequest) with their dictionary indices as sent -- index >= 0 names word i of
 * the global word list, index < 0 names word -index-1 of the message's own Words
 * (mixer/pkg/attribute/dictState.go, protoBag.go:254-266).  Every map field of the message is
 * flattened into CSR arrays: request q's entries of field F are [F_off[q], F_off[q+1]) with keys
 * F_key (attribute-name indices) and the field's values.  Go map keys are unique per message.
 * mxp_wire_decode (mxp.h) turns it into an mxp_bag_batch the way ProtoBag.Get reads it.
 */
typedef struct mxp_wire_batch {
    uint32_t n_requests;
    uint32_t n_global;                 /* global word list (server dictionary)               */
    const uint8_t* global_bytes;
    const uint64_t* global_offsets;    /* [n_global + 1]                                     */
    const uint64_t* words_off;         /* [n + 1] message words of each request:             */
    const uint8_t* word_bytes;         /*   word w spans word_bytes[word_offsets[w] ..       */
    const uint64_t* word_offsets;      /*   word_offsets[w + 1])                             */
    const uint64_t* str_off;   const int32_t* str_key;   const int32_t* str_val;     /* Strings    */
    const uint64_t* i64_off;   const int32_t* i64_key;   const int64_t* i64_val;     /* Int64S     */
    const uint64_t* dbl_off;   const int32_t* dbl_key;   const double* dbl_val;      /* Doubles    */
    const uint64_t* bool_off;  const int32_t* bool_key;  const uint8_t* bool_val;    /* Bools      */
    const uint64_t* ts_off;    const int32_t* ts_key;    const int64_t* ts_sec;      /* Timestamps */
    const int32_t* ts_nsec;
    const uint64_t* dur_off;   const int32_t* dur_key;   const int64_t* dur_val;     /* Durations (ns) */
    const uint64_t* byt_off;   const int32_t* byt_key;                               /* Bytes: entry e */
    const uint64_t* byt_val_off;       /*   spans byt_bytes[byt_val_off[e] .. byt_val_off[e + 1]) */
    const uint8_t* byt_bytes;
    const uint64_t* sm_off;    const int32_t* sm_key;                                /* StringMaps: entry e */
    const uint64_t* sm_ent_off;        /*   has pairs [sm_ent_off[e], sm_ent_off[e + 1]) of   */
    const int32_t* sm_ent_key;         /*   (key, value) word indices                         */
    const int32_t* sm_ent_val;
} mxp_wire_batch;

#ifdef __cplusplus
}
#endif

#endif /* MXP_BATCH_H */
