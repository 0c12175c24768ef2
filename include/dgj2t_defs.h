/*
 * dgj2t_defs.h — the constants of the C ABI (include/dgj2t.h): the
 * reference's j2t flag word, the library's per-message statuses and the API
 * error codes. Split out so the device code includes only these.
 */
#ifndef DGJ2T_DEFS_H
#define DGJ2T_DEFS_H

/* j2t flag bits (reference native/thrift.h:23-32) */
#define DG_F_ALLOW_UNKNOWN (1ull << 0)
#define DG_F_WRITE_DEFAULT (1ull << 1)
#define DG_F_ENABLE_VM (1ull << 2)
#define DG_F_ENABLE_HM (1ull << 3)
#define DG_F_ENABLE_I2S (1ull << 4)
#define DG_F_WRITE_REQUIRE (1ull << 5)
#define DG_F_NO_BASE64 (1ull << 6)
#define DG_F_WRITE_OPTIONAL (1ull << 7)
#define DG_F_TRACE_BACK (1ull << 8)
#define DG_F_NO_WRITE_BASE (1ull << 9)
#define DG_F_VALIDATE_UTF8 (1ull << 16) /* extension: reject invalid UTF-8 in strings */
#define DG_F_NO_FAST_PATH (1ull << 17)  /* extension: run every message on the exact machine (testing) */
#define DG_F_NO_WAVE_PATH (1ull << 18)  /* extension: skip the wave-per-message kernel, lane kernel only (testing) */
#define DG_F_FLAT_PATH (1ull << 19)     /* extension: force the field-major flat kernel (j2t_flat.h) for a flat root
                                           struct (the default whenever the batch's messages are <= 256 B) */
#define DG_F_HM_SPLIT (1ull << 20)      /* extension, with F_ENABLE_HM: the host has already run handleHttpMappings
                                           (conv/j2t/impl.go:243-292) for the ROOT struct; the root raises no ERR_HM,
                                           the mapped fields the host wrote (all of them, or those of the per-message
                                           mask of dg_j2t_batch_*_hm) count as set and their JSON keys are skipped
                                           (native/thrift.c:725), the others are read from the body
                                           (ReadHttpValueFallback). The output is the body part: the host puts its
                                           mapped-field bytes in front. Nested structs with mapped fields still
                                           return ERR_HM. */
#define DG_F_NO_FLAT_PATH (1ull << 21)  /* extension: lane-per-message small kernel even for a flat root (testing) */
#define DG_F_CB_COLLECT (1ull << 22)    /* extension: at a callback the host must serve (ERR_VM_END, a nested
                                           ERR_HM_END, see dg_cb_entry) the machine records it and converts on
                                           instead of stopping; the message ends with DG_ST_CB_LIST and every
                                           callback of one pass recorded, so k callbacks take 2 passes, not k + 1 */

/* library-internal per-message statuses (code byte values the reference never
 * produces). The host entry points resolve them before returning; the device
 * entry point leaves them for the caller and counts them in *d_pending. */
#define DG_ST_OUT_OVERFLOW 0xF0u /* slot too small; out_len = bytes needed (value bits: same, saturated at 2^24-1) */
#define DG_ST_DEEP 0xF1u         /* (internal) nesting beyond the fast kernel's stack */
#define DG_ST_HM_END 0xF2u       /* DG_F_HM_SPLIT + F_TRACE_BACK: the ROOT's ERR_HM_END (native/thrift.c:898-903)
                                    for the host to serve (handleUnmatchedFields, conv/j2t/impl_amd64.go:71-115):
                                    out_len covers the output so far followed by the root's remaining requires
                                    words (big-endian u64, `value` of them); the host appends the cached fields'
                                    bytes and the STOP */
#define DG_ST_HM_END_AT 0xF4u    /* a nested struct's ERR_HM_END for the host (dg_cb_entry) */
#define DG_ST_CB_LIST 0xF5u      /* DG_F_CB_COLLECT: `value` callbacks recorded in the slot, in the order the
                                    message meets them (out_len bytes): each is the status word the stop would
                                    have returned (big-endian u64: code 24 or DG_ST_HM_END_AT, its pos and value)
                                    followed by that stop's record (dg_cb_entry). The host answers them in order
                                    and converts the message again with the answers; an error met after a
                                    callback is reported by that pass, as the reference reports it after Go
                                    served the callback. */
#define DG_ST_HM_ERR 0xF3u       /* DG_F_HM_SPLIT: the message opened a struct whose HTTP-mapping entry is an
                                    error (dg_hm_entry.len == DG_HM_ERR): handleHttpMappings failed for it on the
                                    host; value = the entry's slot, pos = the struct's '{' */

/* HTTP-mapping table of dg_j2t_batch_*_hm: per message, one entry per struct
 * of the descriptor with HTTP-mapped fields (slot j = the j-th such struct in
 * blob order): the bytes the host's handleHttpMappings (conv/j2t/impl.go:
 * 243-292) writes for that struct, at hm_bytes[off, off + len), and the mask
 * of its mapped fields it wrote (bit k = the struct's k-th field in id order;
 * an unset bit = reqs.Set(id, Required), read from the body:
 * ReadHttpValueFallback). len == DG_HM_ERR: the host failed (DG_ST_HM_ERR). */
typedef struct dg_hm_entry {
    uint32_t off;
    uint32_t len;
    uint64_t mask;
} dg_hm_entry;
#define DG_HM_ERR 0xFFFFFFFFu

/* Callbacks the reference returns to its Go host mid-message and resumes
 * after (handleError, conv/j2t/impl_amd64.go:169-247), served here by
 * converting the message again with the host's answers:
 *  - ERR_VM_END (native/thrift.c:641-665): a non-inline value mapping (a
 *    value-mapping type above DG_VM_INLINE_MAX under F_ENABLE_VM; the device
 *    serves DG_VM_BODY_DYNAMIC on a STRING field itself). The host writes the
 *    field header and runs the annotation's ValueMapping.Write on the value's
 *    JSON text (handleValueMapping, impl_amd64.go:117-155).
 *  - ERR_HM_END (native/thrift.c:898-903,952-957) of a NESTED struct under
 *    DG_F_HM_SPLIT + F_TRACE_BACK (the root's is DG_ST_HM_END): the host
 *    writes the cached fields from the request, then STOP
 *    (handleUnmatchedFields, impl_amd64.go:71-115).
 * Per message one dg_cb_entry: `count` answers at bytes[off..], in the order
 * the message meets the callbacks, each a u32 little-endian length and that
 * many bytes. The (count+1)-th callback stops the message:
 *  - ERR_VM_END: status code 24, pos = the value's end (as the reference packs
 *    it); out_len 16: the value's start and the field's descriptor index, two
 *    big-endian u64.
 *  - nested ERR_HM_END: status DG_ST_HM_END_AT (below), value = w, pos = the
 *    position after the '}'; out_len 8 + 8w: the struct's descriptor index,
 *    then w big-endian u64 words whose set bits are the cached fields (bit k =
 *    the struct's k-th field in id order). */
typedef struct dg_cb_entry {
    uint32_t off;
    uint32_t count;
} dg_cb_entry;

/* The host's answers to the reference's Go callbacks for one batch
 * (dg_j2t_batch_*_cb): HTTP-mapping entries (n_hm per message, see
 * dg_hm_entry; hm_tab NULL: none) and callback answers (one dg_cb_entry per
 * message; ans_tab NULL: none), both pointing into `bytes` (len bytes). */
typedef struct dg_cb_tables {
    const dg_hm_entry *hm_tab;
    uint32_t n_hm;
    const dg_cb_entry *ans_tab;
    const uint8_t *bytes;
    uint64_t len;
} dg_cb_tables;

/* API error codes */
#define DG_OK 0
#define DG_E_INVALID (-1)
#define DG_E_HIP (-2)
#define DG_E_NOMEM (-3)
#define DG_E_DESC (-4)
#define DG_E_AGAIN (-5) /* dg_agg_submit(nonblock): no open batch right now */

/* t2j (Thrift binary -> JSON, conv/t2j) option bits: the conv.Options fields
 * conv/t2j/impl.go reads (conv/api.go:52-121) */
#define DG_T2J_BYTE_AS_UINT8 (1ull << 0)     /* ByteAsUint8 */
#define DG_T2J_INT64_AS_STRING (1ull << 1)   /* Int642String */
#define DG_T2J_NULL_FOR_NAN_INF (1ull << 2)  /* EncodeNullJSONForInfOrNan */
#define DG_T2J_NO_BASE64 (1ull << 3)         /* NoBase64Binary */
#define DG_T2J_DISALLOW_UNKNOWN (1ull << 4)  /* DisallowUnknownField */
#define DG_T2J_WRITE_DEFAULT (1ull << 5)     /* WriteDefaultField */
#define DG_T2J_WRITE_REQUIRE (1ull << 6)     /* WriteRequireField */
#define DG_T2J_WRITE_OPTIONAL (1ull << 7)    /* WriteOptionalField */
#define DG_T2J_ENABLE_VM (1ull << 8)         /* EnableValueMapping (api.js_conv, agw.body_dynamic) */
/* the Go-side options, with the host's part done around the kernels
 * (dynamicgo_amd.t2j): */
#define DG_T2J_CONVERT_EXC (1ull << 9)       /* ConvertException: the ROOT struct's first field with a non-zero id
                                                ends the conversion (conv/t2j/impl.go:154-159,173-187): status
                                                DG_T2J_E_EXCEPTION, out = that field's value JSON (then any unset
                                                fields written by handleUnsets) */
#define DG_T2J_HM (1ull << 11)               /* EnableHttpMapping (writeHttpValue, conv/t2j/impl.go:515-588): mapped
                                                fields of the root struct and of its fields' struct values stop for
                                                the host (DG_T2J_E_CALLBACK) */
#define DG_T2J_SKIP_RESP_BASE (1ull << 10)   /* EnableThriftBase with a context BaseResp (readResponseBase,
                                                conv/t2j/impl.go:54-72,120-128): the ROOT's response-base fields
                                                (DG_FF_RESPONSE_BASE) are skipped as STRUCTs, no key written; the
                                                last one's value span [lo, hi) of the message goes to aux as
                                                lo | hi << 32 (~0: none) for the host to FastRead */

/* t2j per-message status codes (bits 0-7 of the status word; pos = Thrift
 * read offset, value as noted). The reference returns Go errors whose
 * meta.ErrorCode behaviour is given. */
#define DG_T2J_E_READ 1           /* ErrRead: truncated input, invalid type / size, skip depth; value = reason */
#define DG_T2J_E_UNKNOWN_FIELD 2  /* ErrUnknownField: value = field id */
#define DG_T2J_E_DISMATCH_TYPE 3  /* ErrDismatchType: value = expected << 8 | got */
#define DG_T2J_E_UNSUPPORTED 4    /* ErrUnsupportedType: value = type */
#define DG_T2J_E_NAN_INF 5        /* ErrWrite: "encounter Nan or Inf double" */
#define DG_T2J_E_MISS_REQUIRED 6  /* ErrMissRequiredField: value = field id */
#define DG_T2J_E_NEEDS_HOST 7     /* a Go-side feature: IDL default JSON values, HTTP mapping, non-inline value mapping,
                                     structs of more than 64 fields */
#define DG_T2J_E_DEPTH 8          /* nesting beyond 4096 containers (the GPU's frame budget; Go recurses further) */
#define DG_T2J_E_WRITE 9          /* ErrWrite: a truncated BYTE/I16/I32/I64/DOUBLE value (doRecurse wraps those reads
                                     as meta.ErrWrite, conv/t2j/impl.go:200-236); value = RD_EOF (1) */
#define DG_T2J_E_EXCEPTION 11     /* DG_T2J_CONVERT_EXC: the exception field's JSON is the output (Go: errors.New(out)) */
#define DG_T2J_E_CALLBACK 12      /* DG_T2J_HM: a writeHttpValue call for the host. out: the payload (the JSON
                                     of a mapped container value, else empty), then a 16-byte trailer of two
                                     little-endian u64: kind (1 a mapped field's value, 2 an unset mapped
                                     field HandleRequires writes) | has-ResponseSetter << 8 | the call's
                                     index << 16 | the field's descriptor index << 32, and the value's start
                                     | its end << 32 (kind 1). The host answers each call (dg_cb_tables
                                     ans_tab, one byte per call in call order: 0 = the response took it, 1 =
                                     write it to the JSON as well, 2 = open: the calls converting its value
                                     follow) and converts the message again. */
#define DG_T2J_E_CONVERT 10       /* ErrConvert: a map key failed (buildinTypeToKey, wrapped as meta.ErrConvert by
                                     conv/t2j/impl.go:355-358): value = the read reason (RD_*), or 0x100 | type for
                                     a key type it does not support */

#endif /* DGJ2T_DEFS_H */
