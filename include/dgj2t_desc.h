/*
 * dgj2t_desc.h — flattened Thrift type-descriptor blob ("dg_desc v1").
 *
 * This is the second input of the j2t hot path. The reference reads its Go
 * descriptor graph in place by mirrored struct layout
 * (reference native/thrift.h:99-137 <-> thrift/descriptor.go:119-267). A GPU
 * cannot chase Go heap pointers, so the host flattens the graph ONCE per
 * descriptor into one position-independent blob of index-linked tables, which
 * is uploaded (or RCCL-broadcast) to every device and then read-only.
 *
 * Layout: a 64-byte header followed by 8-byte-aligned sections. All integers are
 * little-endian. Index fields are u32; DG_NONE marks "absent".
 *
 *   types[n_types]      dg_type    16 B  (ttype, IS_BINARY flag, key/elem/struct links)
 *   structs[n_structs]  dg_struct  32 B
 *   fields[n_fields]    dg_field   24 B  (per struct: contiguous, sorted by field id)
 *   names[n_names]      dg_name    16 B  (per struct: open-addressing table, power of 2)
 *   reqwords[n_reqw]    u64              (per struct: initial requires bits by field INDEX)
 *   pool[pool_len]      bytes            (name keys 8-aligned and zero-padded to a
 *                                         multiple of 8, IDL default-value Thrift bytes)
 *
 * Semantics pinned to the reference:
 *  - field-name lookup = exact match on the key bytes; keys are alias and name,
 *    last Set() wins (internal/util/fieldmap.go:50-62, thrift/idl.go:778-786).
 *    The reference's trie is a lookup accelerator with the same result.
 *  - requires bitmap: the reference keeps one bit per field ID
 *    (thrift/utils.go:30-91, native/map.c:134-154) and walks it in ascending ID
 *    order at '}' (native/thrift.c:258-310). Fields here are sorted by ID, so a
 *    bit per field index walks in the same order; ids that are not fields are
 *    skipped by the reference (f == NULL) and simply have no bit here.
 *  - IS_BINARY = the type's name starts with "binary" (native/thrift.c:1139).
 */
#ifndef DGJ2T_DESC_H
#define DGJ2T_DESC_H

#include <stdint.h>

#define DG_DESC_MAGIC 0x31444744u /* "DGD1" */
#define DG_DESC_VERSION 2u /* v2: alias key per field, 8-aligned keys (v1 blobs still accepted) */
#define DG_NONE 0xffffffffu

/* Thrift wire type codes (reference native/thrift.h:45-63). */
#define DG_T_STOP 0
#define DG_T_VOID 1
#define DG_T_BOOL 2
#define DG_T_BYTE 3
#define DG_T_DOUBLE 4
#define DG_T_I16 6
#define DG_T_I32 8
#define DG_T_I64 10
#define DG_T_STRING 11
#define DG_T_STRUCT 12
#define DG_T_MAP 13
#define DG_T_SET 14
#define DG_T_LIST 15

/* dg_type.flags */
#define DG_TF_BINARY 1u

/* dg_field.required (reference native/map.h:79-81) */
#define DG_REQ_OPTIONAL 0
#define DG_REQ_DEFAULT 1
#define DG_REQ_REQUIRED 2

/* dg_field.flags */
#define DG_FF_REQUEST_BASE 1u /* FieldDescriptor.isRequestBase */
#define DG_FF_HTTP_MAPPING 2u /* len(FieldDescriptor.httpMappings) != 0 */
#define DG_FF_ALIAS_SELF 4u   /* the field's alias key resolves to this field in the name map
                                 (lets the fast path confirm a predicted key by one compare) */
#define DG_FF_KEY_PLAIN 8u    /* the alias has no '"' and no '\\' byte: a JSON key equal to it
                                 ends right after it (no escape can start inside it) */
#define DG_FF_RESPONSE_BASE 16u /* FieldDescriptor.isResponseBase (t2j, EnableThriftBase) */

/* dg_field.vm (reference native/thrift.h:64-67) */
#define DG_VM_NONE 0
#define DG_VM_JSCONV 101
#define DG_VM_INLINE_MAX 255
#define DG_VM_BODY_DYNAMIC 257 /* agw.body_dynamic (thrift/annotation/value_mapping.go:49-51,101-106): the
                                  value's raw JSON text as a Thrift binary; served on the device */

/* dg_struct.flags */
#define DG_SF_HTTP_MAPPING 1u /* len(StructDescriptor.hms) != 0 */

typedef struct dg_desc_hdr {
    uint32_t magic;
    uint32_t version;
    uint32_t total_len;   /* bytes of the whole blob */
    uint32_t root_type;   /* default root type index */
    uint32_t n_types, off_types;
    uint32_t n_structs, off_structs;
    uint32_t n_fields, off_fields;
    uint32_t n_names, off_names;
    uint32_t n_reqwords, off_reqwords;
    uint32_t pool_len, off_pool;
} dg_desc_hdr; /* 64 B */

typedef struct dg_type {
    uint8_t ttype;  /* DG_T_* */
    uint8_t flags;  /* DG_TF_* */
    uint16_t _pad;
    uint32_t key;   /* MAP key type index, else DG_NONE */
    uint32_t elem;  /* LIST/SET/MAP element type index, else DG_NONE */
    uint32_t st;    /* STRUCT index, else DG_NONE */
} dg_type;

typedef struct dg_struct {
    uint32_t field_begin; /* first field (global index); fields sorted by id */
    uint32_t n_fields;
    uint32_t name_begin;  /* first slot of this struct's name table */
    uint32_t name_mask;   /* table size - 1 (size is a power of two, >= 2) */
    uint32_t req_begin;   /* first u64 word of the initial requires bits */
    uint32_t req_words;   /* ceil(n_fields / 64), >= 1 */
    uint32_t flags;       /* DG_SF_* */
    uint32_t _pad;
} dg_struct;

typedef struct dg_field {
    uint16_t id;
    int8_t required;      /* DG_REQ_* (FieldDescriptor.required) */
    uint8_t flags;        /* DG_FF_* */
    uint16_t vm;          /* value-mapping type, DG_VM_* */
    uint16_t key_len;     /* alias key length (bytes) */
    uint32_t type;        /* type index */
    uint32_t dflt_off;    /* pool offset of the IDL default value as Thrift bytes */
    uint32_t dflt_len;    /* DG_NONE = no default value */
    uint32_t key_off;     /* pool offset of the alias key (8-aligned, zero-padded) */
} dg_field;

typedef struct dg_name {
    uint32_t hash;        /* dg_name_hash(key) */
    uint32_t key_off;     /* pool offset */
    uint32_t key_len;
    uint32_t field;       /* global field index, DG_NONE = empty slot */
} dg_name;

/* t2j side table (dg_desc_attach_t2j): per field of the descriptor blob,
 * the JSON text t2j writes for its key, pre-encoded on the host
 * (json.EncodeString(alias) + ':' for fields, EncodeString(name) + ':' for
 * the unset fields handleUnsets writes, conv/t2j/impl.go:150-152,431-433),
 * and the raw alias / name bytes. */
#define DG_T2J_MAGIC 0x32544744u /* "DGT2" */
typedef struct dg_t2j_hdr {
    uint32_t magic;
    uint32_t version;   /* 1 */
    uint32_t total_len;
    uint32_t n_fields;  /* == the descriptor's n_fields */
    uint32_t off_fields;
    uint32_t pool_len, off_pool;
    uint32_t _pad;
} dg_t2j_hdr; /* 32 B */

typedef struct dg_t2j_field {
    uint32_t key_off, key_len;       /* "alias": (quoted, colon) */
    uint32_t name_off, name_len;     /* "name": */
    uint32_t alias_off, alias_len;   /* raw alias bytes */
    uint32_t rname_off, rname_len;   /* raw name bytes */
} dg_t2j_field;

/* Key hash used by the name tables: h = (h * 33) ^ byte, seed 5381. */
#define DG_NAME_HASH_SEED 5381u
#define DG_NAME_HASH_STEP(h, b) ((((h) << 5) + (h)) ^ (uint32_t)(uint8_t)(b))

#endif /* DGJ2T_DESC_H */
