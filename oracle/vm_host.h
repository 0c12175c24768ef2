/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * vm_host.h: the Go host's side of a non-inline value mapping, for the two
 * CPU checkers (oracle/j2t_oracle.c, oracle/ref_harness.c). The reference's
 * FSM stops with ERR_VM_END (native/thrift.c:641-665); Go's handleValueMapping
 * (conv/j2t/impl_amd64.go:117-155) writes the field header and runs the
 * field's ValueMapping.Write on the value's JSON text, then resumes. The
 * mappings restated here are the ones the tests register:
 *   257 agw.body_dynamic   agwBodyDynamic.Write, thrift/annotation/value_mapping.go:101-106
 *   999 test.js_conv2      apiJSConv2.Write, thrift/annotation/value_mapping_test.go:82-111
 * (strconv.ParseInt / ParseFloat restricted to plain decimal text: hex floats
 * and underscores, which Go's ParseFloat also accepts, are rejected here and
 * by the Python mapping the GPU tests register, tests/vm_maps.py).
 */
#pragma once
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define VMH_BODY_DYNAMIC 257
#define VMH_JS_CONV2 999

static inline size_t vmh_be(uint8_t *d, uint64_t v, int k)
{
    for (int i = 0; i < k; i++) d[i] = (uint8_t)(v >> (8 * (k - 1 - i)));
    return (size_t)k;
}

/* strconv.ParseInt(s, 10, 64) on plain decimal text: [+-]?[0-9]+ in range */
static int vmh_parse_int(const uint8_t *s, size_t n, int64_t *out)
{
    size_t i = 0;
    int neg = 0;
    if (i < n && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    if (i == n) return -1;
    uint64_t v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return -1;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return -1;
        v = v * 10 + d;
    }
    if (neg ? v > (uint64_t)1 << 63 : v > (uint64_t)INT64_MAX) return -1; /* ErrRange */
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 0;
}

/* strconv.ParseFloat(s, 64) on plain decimal text
 * [+-]?([0-9]+(\.[0-9]*)?|\.[0-9]+)([eE][+-]?[0-9]+)?; out of range -> error */
static int vmh_parse_float(const uint8_t *s, size_t n, double *out)
{
    size_t i = 0, dg = 0;
    if (i < n && (s[i] == '+' || s[i] == '-')) i++;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++, dg++;
    if (i < n && s[i] == '.') {
        i++;
        while (i < n && s[i] >= '0' && s[i] <= '9') i++, dg++;
    }
    if (!dg) return -1;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        i++;
        if (i < n && (s[i] == '+' || s[i] == '-')) i++;
        size_t e0 = i;
        while (i < n && s[i] >= '0' && s[i] <= '9') i++;
        if (i == e0) return -1;
    }
    if (i != n) return -1;
    char tmp[512];
    if (n >= sizeof tmp) return -1;
    memcpy(tmp, s, n);
    tmp[n] = 0;
    errno = 0;
    double v = strtod(tmp, NULL);
    if (errno == ERANGE && (v > 1.0 || v < -1.0)) return -1; /* overflow: ErrRange (underflow is not an error) */
    *out = v;
    return 0;
}

/* The bytes handleValueMapping appends for field (vm, ftype, fid) with the
 * value text v[0, n): field header (WriteFieldBegin) + Write. dst must hold
 * n + 16 bytes. Returns the length, or -1 if the mapping fails. */
static long vmh_write(uint16_t vm, uint8_t ftype, uint16_t fid, const uint8_t *v, size_t n, uint8_t *dst)
{
    size_t k = 0;
    dst[k++] = ftype;
    k += vmh_be(dst + k, fid, 2);
    if (vm == VMH_BODY_DYNAMIC) {
        if (ftype != 11) return -1; /* "body_dynamic only support STRING type" */
        k += vmh_be(dst + k, n, 4);
        memcpy(dst + k, v, n);
        return (long)(k + n);
    }
    if (vm == VMH_JS_CONV2) {
        if (n == 0) return -1; /* "empty value" */
        if (v[0] == '"') {
            if (n < 2) return -1;
            v += 1;
            n -= 2;
        }
        switch (ftype) {
        case 3: case 6: case 8: case 10: {
            int64_t iv;
            if (vmh_parse_int(v, n, &iv)) return -1;
            /* BinaryProtocol.WriteInt (thrift/binary.go:409-422) */
            k += vmh_be(dst + k, (uint64_t)iv, ftype == 3 ? 1 : ftype == 6 ? 2 : ftype == 8 ? 4 : 8);
            return (long)k;
        }
        case 4: {
            double dv;
            if (vmh_parse_float(v, n, &dv)) return -1;
            uint64_t bits;
            memcpy(&bits, &dv, 8);
            k += vmh_be(dst + k, bits, 8);
            return (long)k;
        }
        default:
            return -1; /* "unsupported type" */
        }
    }
    return -1; /* no mapping registered */
}
