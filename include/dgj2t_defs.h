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

/* library-internal per-message statuses (code byte values the reference never
 * produces). The host entry points resolve them before returning; the device
 * entry point leaves them for the caller and counts them in *d_pending. */
#define DG_ST_OUT_OVERFLOW 0xF0u /* slot too small; out_len = bytes needed (value bits: same, saturated at 2^24-1) */
#define DG_ST_DEEP 0xF1u         /* (internal) nesting beyond the fast kernel's stack */

/* API error codes */
#define DG_OK 0
#define DG_E_INVALID (-1)
#define DG_E_HIP (-2)
#define DG_E_NOMEM (-3)
#define DG_E_DESC (-4)

#endif /* DGJ2T_DEFS_H */
