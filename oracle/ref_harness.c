/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * ref_harness.c: drives the REFERENCE's own C engine, compiled unmodified from
 * where it lies (/root/reference/native/native.c, one translation unit of
 * #includes, reference native/native.c:17-29), behind a tiny C ABI so tests
 * and bench.py's cpu_baseline can call it through ctypes.
 *
 * The harness does only what the reference's Go layer does around the FSM:
 *  - rebuild the reference's descriptor structs (native/thrift.h:70-137) from a
 *    dg_desc v1 blob (include/dgj2t_desc.h): tTypeDesc/tStructDesc/tFieldDesc,
 *    a FieldIdMap indexed by id, a RequiresBitmap by id sized like
 *    thrift/utils.go:30-91, and a TrieTree with no positions whose root leaves
 *    hold every (key, field) pair (trie_get native/map.c:86-132 then does a
 *    linear scan: result-equivalent to the Go-built trie);
 *  - emulate BinaryConv.do (conv/j2t/impl.go:38-91): empty body -> STOP byte,
 *    unquoted STRING root -> json.EncodeString via the reference quote();
 *  - emulate doNative + handleError's OOM re-entry (conv/j2t/impl_amd64.go:
 *    40-69,169-247): grow the buffer / caches and call j2t_fsm_exec again;
 *  - emulate the Do epilogue (conv/j2t/conv.go:70-77): output dropped on error.
 * Inputs are copied into a buffer with a NUL byte after the last byte so the
 * reference's reads of src[len] (e.g. check_leading_zero, native/scanning.c:
 * 781-786) are deterministic; the GPU path defines src[len] == 0 the same way.
 */
#define _GNU_SOURCE 1 /* pthread_setaffinity_np, for the timed CPU baseline */
#include "native.c"

#include <pthread.h>
#include <sched.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dgj2t_desc.h"
#include "../include/dgj2t_defs.h"
#include "vm_host.h"

typedef struct {
    tTypeDesc *types;
    tStructDesc *structs;
    tFieldDesc *fields;
    tFieldDesc ***idbufs;
    uint64_t **reqbufs;
    TrieTree *tries;
    GoSlice *leaves;
    Pair **pairs;
    tDefaultValue *dflts;
    uint32_t n_types, n_structs, n_fields;
    uint8_t *blob;
} RefDesc;

static const char *NAME_BINARY = "binary";
static const char *NAME_OTHER = "other\0\0\0";

void *dgref_desc_create(const uint8_t *blob_in, size_t len)
{
    const dg_desc_hdr *h = (const dg_desc_hdr *)blob_in;
    if (len < sizeof(dg_desc_hdr) || h->magic != DG_DESC_MAGIC || h->total_len > len)
        return NULL;
    RefDesc *d = (RefDesc *)calloc(1, sizeof(RefDesc));
    d->blob = (uint8_t *)malloc(len);
    memcpy(d->blob, blob_in, len);
    const uint8_t *b = d->blob;
    const dg_type *T = (const dg_type *)(b + h->off_types);
    const dg_struct *S = (const dg_struct *)(b + h->off_structs);
    const dg_field *F = (const dg_field *)(b + h->off_fields);
    const dg_name *N = (const dg_name *)(b + h->off_names);
    const uint64_t *R = (const uint64_t *)(b + h->off_reqwords);
    const char *P = (const char *)(b + h->off_pool);
    d->n_types = h->n_types;
    d->n_structs = h->n_structs;
    d->n_fields = h->n_fields;
    d->types = (tTypeDesc *)calloc(h->n_types + 1, sizeof(tTypeDesc));
    d->structs = (tStructDesc *)calloc(h->n_structs + 1, sizeof(tStructDesc));
    d->fields = (tFieldDesc *)calloc(h->n_fields + 1, sizeof(tFieldDesc));
    d->dflts = (tDefaultValue *)calloc(h->n_fields + 1, sizeof(tDefaultValue));
    d->idbufs = (tFieldDesc ***)calloc(h->n_structs + 1, sizeof(void *));
    d->reqbufs = (uint64_t **)calloc(h->n_structs + 1, sizeof(void *));
    d->tries = (TrieTree *)calloc(h->n_structs + 1, sizeof(TrieTree));
    d->leaves = (GoSlice *)calloc(h->n_structs + 1, sizeof(GoSlice));
    d->pairs = (Pair **)calloc(h->n_structs + 1, sizeof(void *));

    for (uint32_t i = 0; i < h->n_types; i++) {
        tTypeDesc *t = &d->types[i];
        t->type = T[i].ttype;
        if (T[i].flags & DG_TF_BINARY) {
            t->name.buf = NAME_BINARY;
            t->name.len = 6;
        } else {
            t->name.buf = NAME_OTHER;
            t->name.len = 5;
        }
        t->key = T[i].key == DG_NONE ? NULL : &d->types[T[i].key];
        t->elem = T[i].elem == DG_NONE ? NULL : &d->types[T[i].elem];
        t->st = T[i].st == DG_NONE ? NULL : &d->structs[T[i].st];
    }
    for (uint32_t i = 0; i < h->n_fields; i++) {
        tFieldDesc *f = &d->fields[i];
        f->is_request_base = (F[i].flags & DG_FF_REQUEST_BASE) != 0;
        f->required = F[i].required;
        f->vm = F[i].vm;
        f->ID = F[i].id;
        f->type = &d->types[F[i].type];
        if (F[i].dflt_len != DG_NONE) {
            d->dflts[i].thrift_binary.buf = P + F[i].dflt_off;
            d->dflts[i].thrift_binary.len = F[i].dflt_len;
            f->default_value = &d->dflts[i];
        }
        /* only len != 0 is read (native/thrift.c:725) */
        f->http_mappings.len = (F[i].flags & DG_FF_HTTP_MAPPING) ? 1 : 0;
    }
    for (uint32_t s = 0; s < h->n_structs; s++) {
        tStructDesc *st = &d->structs[s];
        const dg_struct *ds = &S[s];
        uint32_t maxid = 0;
        for (uint32_t k = 0; k < ds->n_fields; k++)
            if (F[ds->field_begin + k].id > maxid)
                maxid = F[ds->field_begin + k].id;
        /* FieldIDMap: indexed by id */
        size_t idlen = ds->n_fields ? (size_t)maxid + 1 : 0;
        d->idbufs[s] = (tFieldDesc **)calloc(idlen + 1, sizeof(void *));
        for (uint32_t k = 0; k < ds->n_fields; k++)
            d->idbufs[s][F[ds->field_begin + k].id] = &d->fields[ds->field_begin + k];
        st->ids.buf = d->idbufs[s];
        st->ids.len = idlen;
        st->ids.cap = idlen;
        /* RequiresBitmap by id: len = max(len(st.Fields), maxid/64+1) words
         * (thrift/idl.go:679 + RequiresBitmap.Set malloc, thrift/utils.go:46-63) */
        size_t words = ds->n_fields;
        if (ds->n_fields && (size_t)maxid / 64 + 1 > words)
            words = (size_t)maxid / 64 + 1;
        d->reqbufs[s] = (uint64_t *)calloc(words + 1, sizeof(uint64_t));
        for (uint32_t k = 0; k < ds->n_fields; k++) {
            uint64_t w = R[ds->req_begin + k / 64];
            if ((w >> (k % 64)) & 1) {
                uint16_t id = F[ds->field_begin + k].id;
                d->reqbufs[s][id / 64] |= 1ull << (id % 64);
            }
        }
        st->reqs.buf = d->reqbufs[s];
        st->reqs.len = words;
        st->hms.len = (ds->flags & DG_SF_HTTP_MAPPING) ? 1 : 0;
        /* names: trie with zero positions, all pairs in root leaves */
        uint32_t npairs = 0;
        for (uint32_t j = 0; j <= ds->name_mask; j++)
            if (N[ds->name_begin + j].field != DG_NONE)
                npairs++;
        d->pairs[s] = (Pair *)calloc(npairs + 1, sizeof(Pair));
        uint32_t q = 0;
        TrieTree *tr = &d->tries[s];
        for (uint32_t j = 0; j <= ds->name_mask; j++) {
            const dg_name *nm = &N[ds->name_begin + j];
            if (nm->field == DG_NONE)
                continue;
            d->pairs[s][q].val = &d->fields[nm->field];
            d->pairs[s][q].key.buf = P + nm->key_off;
            d->pairs[s][q].key.len = nm->key_len;
            if (nm->key_len == 0)
                tr->empty = &d->fields[nm->field];
            q++;
        }
        d->leaves[s].buf = (char *)d->pairs[s];
        d->leaves[s].len = npairs;
        d->leaves[s].cap = npairs;
        tr->count = npairs;
        tr->node.leaves = &d->leaves[s];
        st->names.trie = npairs ? tr : NULL;
        st->names.hash = NULL;
    }
    return d;
}

void dgref_desc_destroy(void *p)
{
    RefDesc *d = (RefDesc *)p;
    if (!d)
        return;
    for (uint32_t s = 0; s < d->n_structs; s++) {
        free(d->idbufs[s]);
        free(d->reqbufs[s]);
        free(d->pairs[s]);
    }
    free(d->types);
    free(d->structs);
    free(d->fields);
    free(d->dflts);
    free(d->idbufs);
    free(d->reqbufs);
    free(d->tries);
    free(d->leaves);
    free(d->pairs);
    free(d->blob);
    free(d);
}

/* pooled per-thread machine state (internal/types/types.go:313-338) */
typedef struct {
    J2TStateMachine *fsm;
    char *reqs, *keys, *dbuf;
    int32_t *fields;
    size_t reqs_cap, keys_cap, fields_cap;
    char *buf;
    size_t buf_cap;
    char *src;
    size_t src_cap;
} RefCtx;

static RefCtx *ctx_new(void)
{
    RefCtx *c = (RefCtx *)calloc(1, sizeof(RefCtx));
    c->fsm = (J2TStateMachine *)calloc(1, sizeof(J2TStateMachine));
    c->reqs_cap = 1 << 20; /* generous: the OOM re-entry path is exercised only by the reference's own MockConv tests */
    c->keys_cap = 1024;
    c->fields_cap = 4096;
    c->reqs = (char *)malloc(c->reqs_cap);
    c->keys = (char *)malloc(c->keys_cap);
    c->fields = (int32_t *)malloc(c->fields_cap * sizeof(int32_t));
    c->dbuf = (char *)malloc(800);
    return c;
}

static void ctx_free(RefCtx *c)
{
    free(c->fsm);
    free(c->reqs);
    free(c->keys);
    free(c->fields);
    free(c->dbuf);
    free(c->buf);
    free(c->src);
    free(c);
}

static void ensure(char **p, size_t *cap, size_t need)
{
    if (*cap < need) {
        free(*p);
        *cap = need;
        *p = (char *)malloc(need);
    }
}

/* One BinaryConv.Do. Returns the packed reference ret; *out_len = bytes. */
/* handleHttpMappings emulation for the pre-split tests (DG_F_HM_SPLIT): at
 * the ROOT struct's ERR_HM the Go host writes the mapped fields (here: the
 * caller's prefix bytes, as if every value was found) and marks each as set
 * (reqs.Set(id, Optional), conv/j2t/impl.go:243-292), then resumes. */
static const uint8_t *g_hm_prefix;
static size_t g_hm_len;
static int g_hm_on;
/* dgref_j2t_hm2: which mapped fields the host wrote (bit k = the k-th field
 * of the root in id order; the others are reqs.Set(id, Required),
 * ReadHttpValueFallback, conv/j2t/impl.go:276-280), and the root's
 * ERR_HM_END field cache handed back instead of the error */
static uint64_t g_hm_mask = ~0ull;
/* dgref_j2t_hm3: per struct index (blob order) the host's bytes and mask,
 * for an ERR_HM at ANY depth (the bytes handleHttpMappings writes depend on
 * the request and the struct only) */
static const uint8_t *g_hm_bytes;
static const uint32_t *g_hm_off, *g_hm_lens;
static const uint64_t *g_hm_masks;
/* a NESTED struct's ERR_HM_END: the test's host (the Python restatement of
 * handleUnmatchedFields) writes the cached fields + STOP through this
 * callback: (struct index in blob order, field ids, count, dst, cap) ->
 * bytes written, or -1 = the host failed (the ERR_HM_END word is returned) */
typedef long (*dgref_hm_end_fn)(uint32_t, const int32_t *, size_t, uint8_t *, size_t);
static dgref_hm_end_fn g_hm_end_cb;
void dgref_set_hm_end_cb(dgref_hm_end_fn f) { g_hm_end_cb = f; }
static int32_t *g_fc_out;
static size_t g_fc_cap, g_fc_len;
static int g_fc_on;

static uint64_t ref_do(RefCtx *c, RefDesc *d, uint32_t root, const uint8_t *json, size_t n,
                       uint64_t flags, uint8_t *out, size_t out_cap, size_t *out_len)
{
    *out_len = 0;
    const tTypeDesc *desc = &d->types[root];
    if (n == 0) { /* conv/j2t/impl.go:52-82 */
        if (out_cap >= 1)
            out[0] = 0;
        *out_len = 1;
        return 0;
    }
    /* src copy with a NUL sentinel (and quoting for an unquoted STRING root) */
    size_t slen;
    if (desc->type == TTYPE_STRING && json[0] != '"') { /* conv/j2t/impl.go:85-88 */
        ensure(&c->src, &c->src_cap, n * 8 + 16);
        ssize_t dn = n * 8;
        c->src[0] = '"';
        quote((const char *)json, n, c->src + 1, &dn, 0);
        c->src[1 + dn] = '"';
        slen = dn + 2;
    } else {
        ensure(&c->src, &c->src_cap, n + 16);
        memcpy(c->src, json, n);
        slen = n;
    }
    memset(c->src + slen, 0, 8);

    size_t want = slen * 16 + 65536;
    ensure(&c->buf, &c->buf_cap, want);
    GoSlice buf = {c->buf, 0, c->buf_cap - 64 /* b64decode may write past cap */};
    GoString src = {c->src, slen};

    J2TStateMachine *fsm = c->fsm;
    fsm->sp = 1;
    fsm->vt[0].st = 0;
    fsm->vt[0].jp = 0;
    fsm->vt[0].td = desc;
    fsm->reqs_cache.buf = c->reqs;
    fsm->reqs_cache.len = 0;
    fsm->reqs_cache.cap = c->reqs_cap;
    fsm->key_cache.buf = c->keys;
    fsm->key_cache.len = 0;
    fsm->key_cache.cap = c->keys_cap;
    fsm->field_cache.buf = c->fields;
    fsm->field_cache.len = 0;
    fsm->field_cache.cap = c->fields_cap;
    fsm->jt.dbuf = c->dbuf;
    fsm->jt.dcap = 800;

    uint64_t ret;
    for (;;) {
        ret = j2t_fsm_exec(fsm, &buf, &src, flags);
        if (ret == 0)
            break;
        uint8_t e = ret & 0xff;
        size_t p = ret >> 8; /* handleError: int(ret >> ERR_WRAP_SHIFT_CODE) */
        if (e == ERR_OOM_BUF) {
            size_t nc = buf.cap + (buf.cap >> 1);
            if (nc < buf.cap + p)
                nc = buf.cap + p * 2;
            char *nb = (char *)malloc(nc + 64);
            memcpy(nb, buf.buf, buf.len);
            free(c->buf);
            c->buf = nb;
            c->buf_cap = nc + 64;
            buf.buf = nb;
            buf.cap = nc;
            continue;
        }
        if (e == ERR_OOM_BM || e == ERR_OOM_KEY) {
            /* GrowReqCache / GrowKeyCache: a bigger cache; reqs copies live
             * in the old cache are referenced by pointer from the stack, so
             * keep the old block alive (leaked until ctx_free of next call) */
            GoSlice *cs = e == ERR_OOM_BM ? &fsm->reqs_cache : &fsm->key_cache;
            size_t nc = cs->cap * 2 + p;
            char *nb = (char *)malloc(nc);
            memcpy(nb, cs->buf, cs->len);
            /* bitmaps on the stack point into the old cache: rebase them */
            if (e == ERR_OOM_BM) {
                for (size_t i = 0; i < fsm->sp; i++) {
                    J2TState *v = &fsm->vt[i];
                    if (v->td && v->td->type == TTYPE_STRUCT &&
                        (J2T_ST(v->st) == J2T_OBJ || J2T_ST(v->st) == J2T_OBJ_0) &&
                        (char *)v->ex.es.reqs.buf >= cs->buf &&
                        (char *)v->ex.es.reqs.buf < cs->buf + cs->cap)
                        v->ex.es.reqs.buf = (uint64_t *)(nb + ((char *)v->ex.es.reqs.buf - cs->buf));
                }
                free(c->reqs);
                c->reqs = nb;
                c->reqs_cap = nc;
            } else {
                free(c->keys);
                c->keys = nb;
                c->keys_cap = nc;
            }
            cs->buf = nb;
            cs->cap = nc;
            continue;
        }
        if (e == ERR_OOM_FIELD) {
            size_t nc = fsm->field_cache.cap + 4096;
            int32_t *nb = (int32_t *)malloc(nc * sizeof(int32_t));
            memcpy(nb, fsm->field_cache.buf, fsm->field_cache.len * sizeof(int32_t));
            free(c->fields);
            c->fields = nb;
            c->fields_cap = nc;
            fsm->field_cache.buf = nb;
            fsm->field_cache.cap = nc;
            fsm->vt[fsm->sp - 1].jp = p; /* SetPos */
            continue;
        }
        if (e == ERR_HM && g_hm_on && (fsm->sp == 1 || g_hm_off)) {
            J2TState *v = &fsm->vt[fsm->sp - 1];
            const tStructDesc *st = v->td->st;
            if (g_hm_off) {
                const size_t si = (size_t)(st - d->structs);
                if (g_hm_lens[si] == 0xFFFFFFFFu)
                    return ret; /* the host failed for this struct */
                g_hm_prefix = g_hm_bytes + g_hm_off[si];
                g_hm_len = g_hm_lens[si];
                g_hm_mask = g_hm_masks[si];
            }
            for (size_t k = 0, j = 0; k < st->ids.len; k++) {
                const tFieldDesc *f = ((tFieldDesc **)st->ids.buf)[k];
                if (!f)
                    continue;
                if (f->http_mappings.len)
                    bm_set_req(v->ex.es.reqs, f->ID,
                               j >= 64 || ((g_hm_mask >> j) & 1) ? REQ_OPTIONAL : REQ_REQUIRED);
                j++;
            }
            if (buf.len + g_hm_len > buf.cap) {
                size_t nc = (buf.len + g_hm_len) * 2 + 64;
                char *nb = (char *)malloc(nc + 64);
                memcpy(nb, buf.buf, buf.len);
                free(c->buf);
                c->buf = nb;
                c->buf_cap = nc + 64;
                buf.buf = nb;
                buf.cap = nc;
            }
            memcpy(buf.buf + buf.len, g_hm_prefix, g_hm_len);
            buf.len += g_hm_len;
            continue;
        }
        if (e == ERR_HM_END && g_fc_on && fsm->sp == 1) {
            /* the root's unmatched fields: the output so far and the cache,
             * for the caller to serve like handleUnmatchedFields */
            g_fc_len = fsm->field_cache.len;
            for (size_t k = 0; k < g_fc_len && k < g_fc_cap; k++)
                g_fc_out[k] = fsm->field_cache.buf[k];
            *out_len = buf.len;
            if (buf.len <= out_cap)
                memcpy(out, buf.buf, buf.len);
            return ret;
        }
        if (e == ERR_HM_END && g_hm_end_cb && fsm->sp > 1) {
            /* handleError -> handleUnmatchedFields (conv/j2t/impl_amd64.go:71-115,
             * 185-198): the struct on top (At(SP-1)), the field cache, then
             * FieldCache[:0], SP-- and SetPos(pos) */
            const J2TState *sv = &fsm->vt[fsm->sp - 1];
            if (!sv->td || sv->td->type != TTYPE_STRUCT || fsm->field_cache.len == 0)
                break;
            const size_t si = (size_t)(sv->td->st - d->structs);
            uint8_t tmp[1 << 16];
            long k = g_hm_end_cb((uint32_t)si, fsm->field_cache.buf, fsm->field_cache.len, tmp, sizeof tmp);
            if (k < 0)
                break;
            if (buf.len + (size_t)k > buf.cap) {
                size_t nc = (buf.len + (size_t)k) * 2 + 64;
                char *nb = (char *)malloc(nc + 64);
                memcpy(nb, buf.buf, buf.len);
                free(c->buf);
                c->buf = nb;
                c->buf_cap = nc + 64;
                buf.buf = nb;
                buf.cap = nc;
            }
            memcpy(buf.buf + buf.len, tmp, (size_t)k);
            buf.len += (size_t)k;
            fsm->field_cache.len = 0;
            fsm->sp--;
            fsm->vt[fsm->sp - 1].jp = (long)p;
            continue;
        }
        if (e == ERR_VM_END) {
            /* handleError -> handleValueMapping (conv/j2t/impl_amd64.go:117-155,
             * 233-243): the struct at SP-2, the field by id, the value's span from
             * FieldValueCache, field header + ValueMapping.Write, then SP-- and
             * SetPos(pos) (vm_host.h); a failing callback returns the word */
            if (fsm->sp < 2)
                break;
            const J2TState *sv = &fsm->vt[fsm->sp - 2];
            if (!sv->td || sv->td->type != TTYPE_STRUCT)
                break;
            const tStructDesc *st = sv->td->st;
            const FieldVal *fv = &fsm->fval_cache;
            const tFieldDesc *f = (size_t)fv->id < st->ids.len ? ((tFieldDesc **)st->ids.buf)[fv->id] : NULL;
            if (!f || (size_t)fv->end >= slen || fv->start < 0)
                break;
            const size_t vn = (size_t)(fv->end - fv->start);
            if (buf.len + vn + 16 > buf.cap) {
                size_t nc = (buf.len + vn + 16) * 2 + 64;
                char *nb = (char *)malloc(nc + 64);
                memcpy(nb, buf.buf, buf.len);
                free(c->buf);
                c->buf = nb;
                c->buf_cap = nc + 64;
                buf.buf = nb;
                buf.cap = nc;
            }
            long k = vmh_write(f->vm, f->type->type, (uint16_t)f->ID, (const uint8_t *)c->src + fv->start, vn,
                               (uint8_t *)buf.buf + buf.len);
            if (k < 0)
                break;
            buf.len += (size_t)k;
            fsm->sp--;
            if (fsm->sp > 0) {
                fsm->vt[fsm->sp - 1].jp = (long)p;
                continue;
            }
            ret = 0;
            break;
        }
        break; /* real error or host callback (ERR_HM/HM_END) */
    }
    if (ret != 0)
        return ret;
    *out_len = buf.len;
    if (buf.len <= out_cap)
        memcpy(out, buf.buf, buf.len);
    return 0;
}

static RefCtx *g_ctx;

/* one message with the root's HTTP-mapped fields written by the "host" as
 * `prefix` (see g_hm_*); flags should include F_ENABLE_HM */
uint64_t dgref_j2t_hm(void *desc, uint32_t root, const uint8_t *json, size_t n, uint64_t flags,
                      const uint8_t *prefix, size_t plen, uint8_t *out, size_t out_cap, size_t *out_len)
{
    if (!g_ctx)
        g_ctx = ctx_new();
    g_hm_prefix = prefix;
    g_hm_len = plen;
    g_hm_on = 1;
    uint64_t r = ref_do(g_ctx, (RefDesc *)desc, root, json, n, flags, out, out_cap, out_len);
    g_hm_on = 0;
    return r;
}

/* dgref_j2t_hm with the host's per-message mask of written mapped fields;
 * a root ERR_HM_END returns its code with *out_len = the output so far and
 * the field cache in fc[0..*fc_len) */
uint64_t dgref_j2t_hm2(void *desc, uint32_t root, const uint8_t *json, size_t n, uint64_t flags,
                       const uint8_t *prefix, size_t plen, uint64_t mask, uint8_t *out, size_t out_cap,
                       size_t *out_len, int32_t *fc, size_t fc_cap, size_t *fc_len)
{
    if (!g_ctx)
        g_ctx = ctx_new();
    g_hm_prefix = prefix;
    g_hm_len = plen;
    g_hm_on = 1;
    g_hm_mask = mask;
    g_fc_out = fc;
    g_fc_cap = fc_cap;
    g_fc_len = 0;
    g_fc_on = 1;
    uint64_t r = ref_do(g_ctx, (RefDesc *)desc, root, json, n, flags, out, out_cap, out_len);
    g_hm_on = 0;
    g_fc_on = 0;
    g_hm_mask = ~0ull;
    *fc_len = g_fc_len;
    return r;
}

/* dgref_j2t_hm2 with an ERR_HM served at every depth from per-struct
 * entries (index = struct index in blob order; len 0xFFFFFFFF = the host
 * failed: the ERR_HM code is returned) */
uint64_t dgref_j2t_hm3(void *desc, uint32_t root, const uint8_t *json, size_t n, uint64_t flags,
                       const uint8_t *bytes, const uint32_t *off, const uint32_t *len, const uint64_t *masks,
                       uint8_t *out, size_t out_cap, size_t *out_len, int32_t *fc, size_t fc_cap, size_t *fc_len)
{
    g_hm_bytes = bytes;
    g_hm_off = off;
    g_hm_lens = len;
    g_hm_masks = masks;
    uint64_t r = dgref_j2t_hm2(desc, root, json, n, flags, NULL, 0, ~0ull, out, out_cap, out_len, fc, fc_cap, fc_len);
    g_hm_off = NULL;
    g_hm_lens = NULL;
    return r;
}

uint64_t dgref_j2t(void *desc, uint32_t root, const uint8_t *json, size_t n, uint64_t flags,
                   uint8_t *out, size_t out_cap, size_t *out_len)
{
    if (!g_ctx)
        g_ctx = ctx_new();
    return ref_do(g_ctx, (RefDesc *)desc, root, json, n, flags, out, out_cap, out_len);
}

/* ---- batched, multi-threaded driver for the CPU baseline ---- */
typedef struct {
    RefDesc *d;
    uint32_t root;
    const uint8_t *json;
    const uint64_t *in_off;
    uint64_t lo, hi, flags;
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t *out_len;
    uint64_t *ret;
} Job;

static void *run_job(void *arg)
{
    Job *j = (Job *)arg;
    RefCtx *c = ctx_new();
    for (uint64_t i = j->lo; i < j->hi; i++) {
        size_t ol = 0;
        uint64_t cap = j->out_off[i + 1] - j->out_off[i];
        j->ret[i] = ref_do(c, j->d, j->root, j->json + j->in_off[i], j->in_off[i + 1] - j->in_off[i],
                           j->flags, j->out + j->out_off[i], cap, &ol);
        j->out_len[i] = (uint32_t)ol;
    }
    ctx_free(c);
    return NULL;
}

/* Messages [0, n) split into nthreads contiguous byte-balanced shards. */
int dgref_j2t_batch(void *desc, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                    uint64_t n, uint64_t flags, uint8_t *out, const uint64_t *out_off,
                    uint32_t *out_len, uint64_t *ret, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    Job *jobs = (Job *)calloc(nthreads, sizeof(Job));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    uint64_t total = in_off[n] - in_off[0];
    uint64_t lo = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t target = in_off[0] + total * (uint64_t)(t + 1) / nthreads;
        uint64_t hi = lo;
        while (hi < n && (t == nthreads - 1 || in_off[hi] < target))
            hi++;
        jobs[t] = (Job){(RefDesc *)desc, root, json, in_off, lo, hi, flags, out, out_off, out_len, ret};
        lo = hi;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return 0;
}

/* ---- timed driver for bench.py's cpu_baseline (reported baseline only) ----
 * nthreads threads, each pinned to cpus[t] (when given) and owning one
 * contiguous byte-balanced shard, run one untimed warm-up pass (first touch
 * of the caller's preallocated outputs) and then `reps` passes; between
 * passes all threads meet at a barrier, so a pass's time is the slowest
 * shard's. best_s[0]: the best pass in seconds, best_s[1 + r]: pass r. */
typedef struct {
    Job job;
    int cpu, tid, reps;
    pthread_barrier_t *bar;
    double *best;
} TJob;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *run_timed(void *arg)
{
    TJob *t = (TJob *)arg;
    if (t->cpu >= 0) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(t->cpu, &cs);
        pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
    }
    Job *j = &t->job;
    RefCtx *c = ctx_new();
    double t0 = 0;
    for (int r = -1; r < t->reps; r++) {
        pthread_barrier_wait(t->bar);
        if (t->tid == 0)
            t0 = now_s();
        for (uint64_t i = j->lo; i < j->hi; i++) {
            size_t ol = 0;
            uint64_t cap = j->out_off[i + 1] - j->out_off[i];
            j->ret[i] = ref_do(c, j->d, j->root, j->json + j->in_off[i], j->in_off[i + 1] - j->in_off[i],
                               j->flags, j->out + j->out_off[i], cap, &ol);
            j->out_len[i] = (uint32_t)ol;
        }
        pthread_barrier_wait(t->bar);
        if (t->tid == 0 && r >= 0) {
            double dt = now_s() - t0;
            if (t->best[0] < 0 || dt < t->best[0])
                t->best[0] = dt;
            t->best[1 + r] = dt;
        }
    }
    ctx_free(c);
    return NULL;
}

int dgref_j2t_timed(void *desc, uint32_t root, const uint8_t *json, const uint64_t *in_off, uint64_t n,
                    uint64_t flags, uint8_t *out, const uint64_t *out_off, uint32_t *out_len, uint64_t *ret,
                    int nthreads, const int *cpus, int reps, double *best_s)
{
    if (nthreads < 1 || reps < 1 || !best_s)
        return -1;
    TJob *tj = (TJob *)calloc(nthreads, sizeof(TJob));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    best_s[0] = -1;
    uint64_t total = in_off[n] - in_off[0];
    uint64_t lo = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t target = in_off[0] + total * (uint64_t)(t + 1) / nthreads;
        uint64_t hi = lo;
        while (hi < n && (t == nthreads - 1 || in_off[hi] < target))
            hi++;
        tj[t].job = (Job){(RefDesc *)desc, root, json, in_off, lo, hi, flags, out, out_off, out_len, ret};
        tj[t].cpu = cpus ? cpus[t] : -1;
        tj[t].tid = t;
        tj[t].reps = reps;
        tj[t].bar = &bar;
        tj[t].best = best_s;
        lo = hi;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, run_timed, &tj[t]);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    free(tj);
    free(th);
    return 0;
}

/* ====================================================================== */
/* t2j (Thrift binary -> JSON): a C restatement of the reference's Go t2j  */
/* (conv/t2j/impl.go:74-607, thrift/binary.go read functions,              */
/* thrift/binary_skip.go:105-210 skipType, thrift/utils.go:149-176         */
/* HandleRequires, thrift/annotation/value_mapping.go:143-214 js_conv Read)*/
/* over the reference's OWN native encoders compiled above: quote()        */
/* (native/parsing.c:487), i64toa (native/fastint.c:212), f64toa           */
/* (native/fastfloat.c:349) and b64encode (native/base64.c:173). The Go    */
/* control flow is restated (no Go toolchain here); the byte encoders are  */
/* the reference's.                                                        */
/* ====================================================================== */
typedef struct {
    const uint8_t *b;
    size_t n, p;
} TRd;
typedef struct {
    char *b;
    size_t len, cap;
} JBuf;
typedef struct {
    const uint8_t *blob;
    const dg_desc_hdr *h;
    const dg_type *T;
    const dg_struct *S;
    const dg_field *F;
    const uint64_t *R;
    const dg_t2j_field *X;
    const char *XP; /* side-table pool */
    uint64_t opts;
    uint64_t *aux; /* DG_T2J_SKIP_RESP_BASE: the base field's span (lo | hi << 32) */
    /* DG_T2J_HM: the host's answers to writeHttpValue calls, in call order
     * (0 taken, 1 write to the JSON too, 2 open), and the calls so far */
    const uint8_t *ans;
    uint32_t n_ans;
    uint32_t *seen;
} T2J;

#define T2J_ERR(code, pos, val) ((uint64_t)(code) | ((uint64_t)(pos) << 8) | ((uint64_t)(val) << 40))
enum { RD_EOF = 1, RD_BAD_TYPE = 2, RD_BAD_SIZE = 3, RD_DEPTH = 4 };

static void jb_reserve(JBuf *o, size_t k)
{
    if (o->len + k + 64 > o->cap) {
        size_t nc = (o->cap + k + 64) * 2;
        char *nb = (char *)malloc(nc);
        memcpy(nb, o->b, o->len);
        free(o->b);
        o->b = nb;
        o->cap = nc;
    }
}
static void jb_put(JBuf *o, const void *s, size_t k)
{
    jb_reserve(o, k);
    memcpy(o->b + o->len, s, k);
    o->len += k;
}
static void jb_c(JBuf *o, char c) { jb_put(o, &c, 1); }
static void jb_i64(JBuf *o, int64_t v)
{
    jb_reserve(o, 32);
    o->len += (size_t)i64toa(o->b + o->len, v); /* native/fastint.c:212 */
}
static void jb_f64(JBuf *o, double v)
{
    jb_reserve(o, 40);
    o->len += (size_t)f64toa(o->b + o->len, v); /* native/fastfloat.c:349 (0 for inf/nan: nothing, like the Go wrapper) */
}
static void jb_quote(JBuf *o, const uint8_t *s, size_t n) /* json.NoQuote: native quote, flags 0 */
{
    if (!n)
        return;
    ssize_t dn = (ssize_t)(n * 6 + 8);
    jb_reserve(o, (size_t)dn);
    quote((const char *)s, (ssize_t)n, o->b + o->len, &dn, 0);
    o->len += (size_t)dn;
}
static void jb_string(JBuf *o, const uint8_t *s, size_t n) /* json.EncodeString */
{
    jb_c(o, '"');
    jb_quote(o, s, n);
    jb_c(o, '"');
}

static int rd_need(TRd *r, size_t k) { return r->p + k <= r->n; }
static uint64_t rd_be(TRd *r, int k)
{
    uint64_t v = 0;
    for (int i = 0; i < k; i++)
        v = (v << 8) | r->b[r->p + i];
    r->p += (size_t)k;
    return v;
}
static int ttype_valid(uint8_t t) /* thrift/descriptor.go:60-67 */
{
    switch (t) {
    case 0: case 1: case 2: case 3: case 4: case 6: case 8: case 10: case 11: case 12: case 13: case 14: case 15:
    case 16: case 17:
        return 1;
    }
    return 0;
}
static int fixed_size(uint8_t t) /* typeSize, thrift/binary_skip.go:26-41 */
{
    switch (t) {
    case 2: case 3: return 1;
    case 6: return 2;
    case 8: return 4;
    case 10: case 4: return 8;
    }
    return 0;
}

/* skipstr (thrift/binary_skip.go:80-95): the size is read as uint32 into a
 * 64-bit int; nothing is consumed on failure */
static int t2j_skipstr(TRd *r)
{
    if (!rd_need(r, 4)) return RD_EOF;
    uint64_t sz = ((uint64_t)r->b[r->p] << 24) | ((uint64_t)r->b[r->p + 1] << 16) | ((uint64_t)r->b[r->p + 2] << 8) |
                  r->b[r->p + 3];
    if (r->p + 4 + sz > r->n) return RD_EOF;
    r->p += 4 + sz;
    return 0;
}

/* skipType (thrift/binary_skip.go:109-210): 0 or an RD_* reason */
static int t2j_skip(TRd *r, uint8_t t, int depth)
{
    if (depth <= 0)
        return RD_DEPTH;
    int fs = fixed_size(t);
    if (fs > 0) {
        if (!rd_need(r, (size_t)fs)) return RD_EOF;
        r->p += (size_t)fs;
        return 0;
    }
    switch (t) {
    case 11:
        return t2j_skipstr(r);
    case 12:
        for (;;) {
            if (!rd_need(r, 1)) return RD_EOF;
            uint8_t tp = r->b[r->p++];
            if (tp == 0) break;
            if (!rd_need(r, 2)) return RD_EOF;
            r->p += 2;
            int e = fixed_size(tp) > 0 ? (rd_need(r, (size_t)fixed_size(tp)) ? (r->p += (size_t)fixed_size(tp), 0) : RD_EOF)
                                       : t2j_skip(r, tp, depth - 1);
            if (e) return e;
        }
        return 0;
    case 13: {
        if (!rd_need(r, 6)) return RD_EOF;
        uint8_t kt = r->b[r->p], vt = r->b[r->p + 1];
        r->p += 2;
        int32_t sz = (int32_t)rd_be(r, 4);
        if (sz < 0) return RD_BAD_SIZE;
        int ks = fixed_size(kt), vs = fixed_size(vt);
        if (ks > 0 && vs > 0) {
            uint64_t k = (uint64_t)sz * (uint64_t)(ks + vs);
            if (!rd_need(r, k)) return RD_EOF;
            r->p += k;
            return 0;
        }
        for (int32_t i = 0; i < sz; i++) {
            int e;
            if (ks > 0) e = rd_need(r, (size_t)ks) ? (r->p += (size_t)ks, 0) : RD_EOF;
            else e = kt == 11 ? t2j_skipstr(r) : t2j_skip(r, kt, depth - 1);
            if (e) return e;
            if (vs > 0) e = rd_need(r, (size_t)vs) ? (r->p += (size_t)vs, 0) : RD_EOF;
            else e = vt == 11 ? t2j_skipstr(r) : t2j_skip(r, vt, depth - 1);
            if (e) return e;
        }
        return 0;
    }
    case 14: case 15: {
        if (!rd_need(r, 5)) return RD_EOF;
        uint8_t vt = r->b[r->p++];
        int32_t sz = (int32_t)rd_be(r, 4);
        if (sz < 0) return RD_BAD_SIZE;
        int vs = fixed_size(vt);
        if (vs > 0) {
            uint64_t k = (uint64_t)sz * (uint64_t)vs;
            if (!rd_need(r, k)) return RD_EOF;
            r->p += k;
            return 0;
        }
        for (int32_t i = 0; i < sz; i++) {
            int e = vt == 11 ? t2j_skipstr(r) : t2j_skip(r, vt, depth - 1);
            if (e) return e;
        }
        return 0;
    }
    }
    return RD_BAD_SIZE; /* default: errInvalidDataSize */
}

static int32_t t2j_field_by_id(const T2J *c, const dg_struct *sd, uint16_t id)
{
    for (uint32_t k = 0; k < sd->n_fields; k++)
        if (c->F[sd->field_begin + k].id == id)
            return (int32_t)(sd->field_begin + k);
    return -1;
}

static uint64_t t2j_value_r(const T2J *c, uint32_t td, TRd *r, JBuf *o, int resp);
static uint64_t t2j_value(const T2J *c, uint32_t td, TRd *r, JBuf *o) { return t2j_value_r(c, td, r, o, 0); }

/* a writeHttpValue call the host must make (DG_T2J_E_CALLBACK): the record
 * after the payload already in o, as include/dgj2t_defs.h lays it out */
static uint64_t t2j_stop(TRd *r, JBuf *o, uint32_t kind, uint32_t idx, uint32_t fi, size_t s0, size_t s1)
{
    if (idx > 0xFFFF) return T2J_ERR(DG_T2J_E_DEPTH, r->p, idx);
    uint64_t w[2] = {(uint64_t)kind | ((uint64_t)idx << 16) | ((uint64_t)fi << 32),
                     (uint64_t)(uint32_t)s0 | ((uint64_t)(uint32_t)s1 << 32)};
    jb_put(o, w, 16);
    return T2J_ERR(DG_T2J_E_CALLBACK, r->p, kind & 0xFF);
}

/* writeDefaultOrEmpty (conv/t2j/impl.go:440-468) */
static uint64_t t2j_default_or_empty(const T2J *c, const dg_field *f, size_t pos, JBuf *o)
{
    if (f->dflt_len != DG_NONE) {
        /* DefaultValue().JSONValue() (thrift/idl.go:834-955) of a scalar or
         * string constant, from its Thrift bytes; containers stay Go-side */
        const uint8_t *b = c->blob + c->h->off_pool + f->dflt_off;
        const uint8_t tt = c->T[f->type].ttype;
        uint64_t u = 0;
        int nb = tt == 3 ? 1 : tt == 6 ? 2 : tt == 8 ? 4 : (tt == 10 || tt == 4) ? 8 : 0;
        for (int k = 0; k < nb; k++) u = (u << 8) | b[k];
        switch (tt) {
        case 2: if (b[0] == 1) jb_put(o, "true", 4); else jb_put(o, "false", 5); return 0;
        case 3: jb_i64(o, (int8_t)u); return 0;
        case 6: jb_i64(o, (int16_t)u); return 0;
        case 8: jb_i64(o, (int32_t)u); return 0;
        case 10: jb_i64(o, (int64_t)u); return 0;
        case 4: { double d; memcpy(&d, &u, 8); jb_f64(o, d); return 0; }
        case 11: {
            uint32_t n = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
            jb_string(o, b + 4, n);
            return 0;
        }
        }
        return T2J_ERR(DG_T2J_E_NEEDS_HOST, pos, f->id); /* a container constant: Go-side */
    }
    switch (c->T[f->type].ttype) {
    case 2: jb_put(o, "false", 5); return 0;
    case 3: case 6: case 8: case 10: jb_i64(o, 0); return 0;
    case 4: jb_f64(o, 0.0); return 0;
    case 11: jb_put(o, "\"\"", 2); return 0;
    case 14: case 15: jb_put(o, "[]", 2); return 0;
    case 13: jb_put(o, "{}", 2); return 0;
    case 12: jb_put(o, "{}", 2); return 0;
    }
    return T2J_ERR(DG_T2J_E_UNSUPPORTED, pos, c->T[f->type].ttype);
}

/* js_conv Read (thrift/annotation/value_mapping.go:143-214): appendInt */
static uint64_t t2j_append_int(const T2J *c, uint8_t t, TRd *r, JBuf *o)
{
    jb_c(o, '"');
    switch (t) {
    case 3: if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF); jb_i64(o, (int64_t)(uint8_t)rd_be(r, 1)); break;
    case 6: if (!rd_need(r, 2)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF); jb_i64(o, (int16_t)rd_be(r, 2)); break;
    case 8: if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF); jb_i64(o, (int32_t)rd_be(r, 4)); break;
    case 10: if (!rd_need(r, 8)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF); jb_i64(o, (int64_t)rd_be(r, 8)); break;
    case 4: {
        if (!rd_need(r, 8)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint64_t u = rd_be(r, 8);
        double d;
        memcpy(&d, &u, 8);
        jb_f64(o, d);
        break;
    }
    case 11: {
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t sz = (int32_t)rd_be(r, 4);
        if (sz < 0 || !rd_need(r, (size_t)sz)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        jb_put(o, r->b + r->p, (size_t)sz); /* raw, not escaped */
        r->p += (size_t)sz;
        break;
    }
    default:
        return T2J_ERR(DG_T2J_E_UNSUPPORTED, r->p, t);
    }
    jb_c(o, '"');
    return 0;
}

static uint64_t t2j_vm(const T2J *c, const dg_field *f, TRd *r, JBuf *o)
{
    if (f->vm == DG_VM_BODY_DYNAMIC) { /* agwBodyDynamic.Read (thrift/annotation/value_mapping.go:84-99) */
        if (c->T[f->type].ttype != 11) return T2J_ERR(DG_T2J_E_CONVERT, r->p, 0x200u | c->T[f->type].ttype);
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t sz = (int32_t)rd_be(r, 4);
        if (sz < 0 || !rd_need(r, (size_t)sz)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        jb_put(o, r->b + r->p, (size_t)sz); /* the raw bytes are the JSON */
        r->p += (size_t)sz;
        return 0;
    }
    if (f->vm != DG_VM_JSCONV)
        return T2J_ERR(DG_T2J_E_NEEDS_HOST, r->p, f->vm);
    if (c->T[f->type].ttype == 15) { /* LIST: ReadListBegin, elements by the wire type */
        jb_c(o, '[');
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF); /* ReadListBegin */
        uint8_t et = r->b[r->p++];
        if (!ttype_valid(et)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_TYPE);
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t n = (int32_t)rd_be(r, 4);
        if (n < 0) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        for (int32_t i = 0; i < n; i++) {
            uint64_t e = t2j_append_int(c, et, r, o);
            if (e) return e;
            if (i != n - 1) jb_c(o, ',');
        }
        jb_c(o, ']');
        return 0;
    }
    return t2j_append_int(c, c->T[f->type].ttype, r, o);
}

/* a STRUCT value (conv/t2j/impl.go:265-339); top: the root struct (do(),
 * impl.go:74-187): response-base fields skipped (readResponseBase, the span
 * to c->aux) and the exception field (ConvertException) ending it. resp: a
 * ResponseSetter is passed here (the root, a root field's struct value, a
 * value writeHttpValue converts): its mapped fields go to writeHttpValue
 * (impl.go:132-142, 296-306), the Go host's part, asked for by a stop. */
static uint64_t t2j_struct_at(const T2J *c, uint32_t td, TRd *r, JBuf *o, int top, int resp)
{
    const dg_struct *sd = &c->S[c->T[td].st];
    jb_c(o, '{');
    uint64_t req[64];
    uint32_t nw = sd->req_words < 64 ? sd->req_words : 64;
    for (uint32_t w = 0; w < nw; w++)
        req[w] = c->R[sd->req_begin + w];
    int comma = 0, exc_done = 0;
    for (;;) {
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint8_t t = r->b[r->p++];
        if (!ttype_valid(t)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_TYPE);
        if (t == 0) break;
        if (!rd_need(r, 2)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint16_t id = (uint16_t)rd_be(r, 2);
        int32_t fi = t2j_field_by_id(c, sd, id);
        if (fi < 0) {
            if (c->opts & DG_T2J_DISALLOW_UNKNOWN) return T2J_ERR(DG_T2J_E_UNKNOWN_FIELD, r->p, id);
            int e = t2j_skip(r, t, 1023);
            if (e) return T2J_ERR(DG_T2J_E_READ, r->p, e);
            continue;
        }
        const dg_field *f = &c->F[fi];
        uint32_t k = (uint32_t)fi - sd->field_begin;
        req[k / 64] &= ~(1ull << (k % 64)); /* r.Set(id, Optional) */
        if (top && (c->opts & DG_T2J_SKIP_RESP_BASE) && (f->flags & DG_FF_RESPONSE_BASE)) {
            size_t s0 = r->p; /* readResponseBase: SkipType(STRUCT), the bytes to base.FastRead */
            int se = t2j_skip(r, 12, 1023);
            if (se) return T2J_ERR(DG_T2J_E_READ, r->p, se);
            if (c->aux) *c->aux = (uint64_t)s0 | ((uint64_t)r->p << 32);
            continue;
        }
        if ((c->opts & DG_T2J_HM) && resp && (f->flags & DG_FF_HTTP_MAPPING)) {
            const uint32_t idx = (*c->seen)++;
            const int a = idx < c->n_ans ? c->ans[idx] : 2;
            const uint8_t dt = c->T[f->type].ttype;
            if (idx >= c->n_ans) { /* a new call: the host reads the value at r->p */
                o->len = 0;
                return t2j_stop(r, o, 1 | 0x100u, idx, (uint32_t)fi, r->p, r->p);
            }
            if (a == 2 && (dt == 12 || dt == 13 || dt == 14 || dt == 15)) {
                /* the call needs the container's JSON (doRecurse(resp), impl.go:561-574) */
                size_t s0 = r->p;
                o->len = 0;
                uint64_t e = t2j_value_r(c, f->type, r, o, 1);
                if (e) return e;
                return t2j_stop(r, o, 1 | 0x100u, idx, (uint32_t)fi, s0, r->p);
            }
            if (a == 0) { /* the response took it (!WriteHttpValueFallback || ok) */
                int se = t2j_skip(r, dt, 1023);
                if (se) return T2J_ERR(DG_T2J_E_READ, r->p, se);
                continue;
            }
        }
        if (comma) jb_c(o, ',');
        else comma = 1;
        const dg_t2j_field *x = &c->X[fi];
        jb_string(o, (const uint8_t *)c->XP + x->alias_off, x->alias_len);
        jb_c(o, ':');
        const int exc = top && (c->opts & DG_T2J_CONVERT_EXC) && id != 0;
        if (exc) o->len = 0; /* only the exception field's data */
        uint64_t e;
        if ((c->opts & DG_T2J_ENABLE_VM) && f->vm != DG_VM_NONE) e = t2j_vm(c, f, r, o);
        else e = t2j_value_r(c, f->type, r, o, top && resp); /* do() passes resp on (impl.go:167) */
        if (e) return e;
        if (exc) {
            exc_done = 1;
            break;
        }
    }
    /* handleUnsets -> HandleRequires (thrift/utils.go:149-176), ascending id */
    for (uint32_t k = 0; k < sd->n_fields; k++) {
        if (!((req[k / 64] >> (k % 64)) & 1)) continue;
        const dg_field *f = &c->F[sd->field_begin + k];
        if (f->required == DG_REQ_REQUIRED && !(c->opts & DG_T2J_WRITE_REQUIRE))
            return T2J_ERR(DG_T2J_E_MISS_REQUIRED, r->p, f->id);
        if ((f->required == DG_REQ_DEFAULT && !(c->opts & DG_T2J_WRITE_DEFAULT)) ||
            (f->required == DG_REQ_OPTIONAL && !(c->opts & DG_T2J_WRITE_OPTIONAL) && f->dflt_len == DG_NONE))
            continue;
        if ((c->opts & DG_T2J_HM) && (f->flags & DG_FF_HTTP_MAPPING)) {
            /* handleUnsets (impl.go:401-429): writeHttpValue of the default first */
            const uint32_t idx = (*c->seen)++;
            if (idx >= c->n_ans) {
                o->len = 0;
                return t2j_stop(r, o, 2 | (resp ? 0x100u : 0u), idx, sd->field_begin + k, 0, 0);
            }
            if (c->ans[idx] == 0) continue;
        }
        if (comma) jb_c(o, ','); /* EncodeArrayComma */
        else comma = 1;
        const dg_t2j_field *x = &c->X[sd->field_begin + k];
        jb_string(o, (const uint8_t *)c->XP + x->rname_off, x->rname_len); /* field.Name() */
        jb_c(o, ':');
        uint64_t e = t2j_default_or_empty(c, f, r->p, o);
        if (e) return e;
    }
    if (exc_done) return T2J_ERR(DG_T2J_E_EXCEPTION, r->p, 0); /* err = errors.New(string(*out)) */
    jb_c(o, '}');
    return 0;
}

/* doRecurse (conv/t2j/impl.go:189-393); resp reaches a STRUCT only */
static uint64_t t2j_value_r(const T2J *c, uint32_t td, TRd *r, JBuf *o, int resp)
{
    const dg_type *t = &c->T[td];
    switch (t->ttype) {
    case 2: {
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        if (r->b[r->p++] == 1) jb_put(o, "true", 4);
        else jb_put(o, "false", 5);
        return 0;
    }
    case 3: {
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_WRITE, r->p, RD_EOF);
        uint8_t v = r->b[r->p++];
        jb_i64(o, (c->opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
        return 0;
    }
    case 6:
        if (!rd_need(r, 2)) return T2J_ERR(DG_T2J_E_WRITE, r->p, RD_EOF);
        jb_i64(o, (int16_t)rd_be(r, 2));
        return 0;
    case 8:
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_WRITE, r->p, RD_EOF);
        jb_i64(o, (int32_t)rd_be(r, 4));
        return 0;
    case 10:
        if (!rd_need(r, 8)) return T2J_ERR(DG_T2J_E_WRITE, r->p, RD_EOF);
        if (c->opts & DG_T2J_INT64_AS_STRING) {
            jb_c(o, '"');
            jb_i64(o, (int64_t)rd_be(r, 8));
            jb_c(o, '"');
        } else {
            jb_i64(o, (int64_t)rd_be(r, 8));
        }
        return 0;
    case 4: {
        if (!rd_need(r, 8)) return T2J_ERR(DG_T2J_E_WRITE, r->p, RD_EOF);
        uint64_t u = rd_be(r, 8);
        if (((u >> 52) & 0x7FF) == 0x7FF) { /* NaN or Inf */
            if (!(c->opts & DG_T2J_NULL_FOR_NAN_INF)) return T2J_ERR(DG_T2J_E_NAN_INF, r->p, 0);
            jb_put(o, "null", 4);
            return 0;
        }
        double d;
        memcpy(&d, &u, 8);
        jb_f64(o, d);
        return 0;
    }
    case 11: {
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t sz = (int32_t)rd_be(r, 4);
        if (sz < 0 || !rd_need(r, (size_t)sz)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        const uint8_t *s = r->b + r->p;
        r->p += (size_t)sz;
        if ((t->flags & DG_TF_BINARY) && !(c->opts & DG_T2J_NO_BASE64)) { /* EncodeBaniry */
            jb_c(o, '"');
            if (sz) {
                size_t cap = ((size_t)sz + 2) / 3 * 4 + 8;
                jb_reserve(o, cap);
                GoSlice out = {o->b + o->len, 0, (ssize_t)cap};
                GoSlice src = {(char *)s, sz, sz};
                b64encode(&out, &src, 0); /* std alphabet, padded (base64x.StdEncoding) */
                o->len += ((size_t)sz + 2) / 3 * 4;
            }
            jb_c(o, '"');
        } else {
            jb_string(o, s, (size_t)sz);
        }
        return 0;
    }
    case 12:
        return t2j_struct_at(c, td, r, o, 0, resp);
    case 13: {
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint8_t kt = r->b[r->p++];
        if (!ttype_valid(kt)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_TYPE);
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint8_t vt = r->b[r->p++];
        if (!ttype_valid(vt)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_TYPE);
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t n = (int32_t)rd_be(r, 4);
        if (n < 0) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        const dg_type *K = &c->T[t->key], *V = &c->T[t->elem];
        if (kt != K->ttype) return T2J_ERR(DG_T2J_E_DISMATCH_TYPE, r->p, ((uint32_t)K->ttype << 8) | kt);
        if (vt != V->ttype) return T2J_ERR(DG_T2J_E_DISMATCH_TYPE, r->p, ((uint32_t)V->ttype << 8) | vt);
        jb_c(o, '{');
        for (int32_t i = 0; i < n; i++) {
            if (i) jb_c(o, ',');
            jb_c(o, '"'); /* buildinTypeToKey (conv/t2j/impl.go:470-530) */
            switch (K->ttype) {
            case 3: {
                if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_EOF);
                uint8_t v = r->b[r->p++];
                jb_i64(o, (c->opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
                break;
            }
            case 6: if (!rd_need(r, 2)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_EOF); jb_i64(o, (int16_t)rd_be(r, 2)); break;
            case 8: if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_EOF); jb_i64(o, (int32_t)rd_be(r, 4)); break;
            case 10: if (!rd_need(r, 8)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_EOF); jb_i64(o, (int64_t)rd_be(r, 8)); break;
            case 11: {
                if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_EOF);
                int32_t sz = (int32_t)rd_be(r, 4);
                if (sz < 0 || !rd_need(r, (size_t)sz)) return T2J_ERR(DG_T2J_E_CONVERT, r->p, RD_BAD_SIZE);
                jb_quote(o, r->b + r->p, (size_t)sz);
                r->p += (size_t)sz;
                break;
            }
            default:
                return T2J_ERR(DG_T2J_E_CONVERT, r->p, 0x100u | K->ttype); /* conv/t2j/impl.go:355-358 */
            }
            jb_c(o, '"');
            jb_c(o, ':');
            uint64_t e = t2j_value(c, t->elem, r, o);
            if (e) return e;
        }
        jb_c(o, '}');
        return 0;
    }
    case 14: case 15: {
        if (!rd_need(r, 1)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        uint8_t et = r->b[r->p++];
        if (!ttype_valid(et)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_TYPE);
        if (!rd_need(r, 4)) return T2J_ERR(DG_T2J_E_READ, r->p, RD_EOF);
        int32_t n = (int32_t)rd_be(r, 4);
        if (n < 0) return T2J_ERR(DG_T2J_E_READ, r->p, RD_BAD_SIZE);
        const dg_type *E = &c->T[t->elem];
        if (et != E->ttype) return T2J_ERR(DG_T2J_E_DISMATCH_TYPE, r->p, ((uint32_t)E->ttype << 8) | et);
        jb_c(o, '[');
        for (int32_t i = 0; i < n; i++) {
            if (i) jb_c(o, ',');
            uint64_t e = t2j_value(c, t->elem, r, o);
            if (e) return e;
        }
        jb_c(o, ']');
        return 0;
    }
    }
    return T2J_ERR(DG_T2J_E_UNSUPPORTED, r->p, t->ttype);
}

static void t2j_init(T2J *c, const uint8_t *blob, const uint8_t *side, uint64_t opts)
{
    c->blob = blob;
    c->h = (const dg_desc_hdr *)blob;
    c->T = (const dg_type *)(blob + c->h->off_types);
    c->S = (const dg_struct *)(blob + c->h->off_structs);
    c->F = (const dg_field *)(blob + c->h->off_fields);
    c->R = (const uint64_t *)(blob + c->h->off_reqwords);
    const dg_t2j_hdr *xh = (const dg_t2j_hdr *)side;
    c->X = (const dg_t2j_field *)(side + xh->off_fields);
    c->XP = (const char *)(side + xh->off_pool);
    c->opts = opts & ~(uint64_t)DG_T2J_HM; /* dgref_t2j3 only: it has the answers */
    c->aux = NULL;
    c->ans = NULL;
    c->n_ans = 0;
    c->seen = NULL;
}

/* BinaryConv.Do (conv/t2j/conv.go:50-75 + impl.go:74-187): one message into
 * o (reset first; the caller's buffer is reused like conv.NewBytes' pool).
 * Returns the status word; on success the JSON is o->b[0, o->len). */
static uint64_t t2j_do(const T2J *c, uint32_t root, const uint8_t *thrift, size_t n, JBuf *o)
{
    TRd r = {thrift, n, 0};
    o->len = 0;
    if (c->aux) *c->aux = ~0ull;
    if (c->seen) *c->seen = 0;
    if (c->T[root].ttype == 12) return t2j_struct_at(c, root, &r, o, 1, (c->opts & DG_T2J_HM) != 0);
    return t2j_value(c, root, &r, o);
}

uint64_t dgref_t2j(const uint8_t *blob, const uint8_t *side, uint32_t root, const uint8_t *thrift, size_t n,
                   uint64_t opts, uint8_t *out, size_t cap, size_t *out_len)
{
    T2J c;
    t2j_init(&c, blob, side, opts);
    JBuf o = {(char *)malloc(256), 0, 256};
    uint64_t e = t2j_do(&c, root, thrift, n, &o);
    const int keep = !e || (e & 0xFF) == DG_T2J_E_EXCEPTION;
    *out_len = keep ? o.len : 0;
    if (keep && o.len <= cap)
        memcpy(out, o.b, o.len);
    free(o.b);
    return e;
}

/* dgref_t2j with the response-base span (DG_T2J_SKIP_RESP_BASE) */
uint64_t dgref_t2j2(const uint8_t *blob, const uint8_t *side, uint32_t root, const uint8_t *thrift, size_t n,
                    uint64_t opts, uint8_t *out, size_t cap, size_t *out_len, uint64_t *aux)
{
    T2J c;
    t2j_init(&c, blob, side, opts);
    c.aux = aux;
    JBuf o = {(char *)malloc(256), 0, 256};
    uint64_t e = t2j_do(&c, root, thrift, n, &o);
    const int keep = !e || (e & 0xFF) == DG_T2J_E_EXCEPTION;
    *out_len = keep ? o.len : 0;
    if (keep && o.len <= cap)
        memcpy(out, o.b, o.len);
    free(o.b);
    return e;
}

/* dgref_t2j2 with the host's writeHttpValue answers (DG_T2J_HM); a
 * DG_T2J_E_CALLBACK keeps its record in out */
uint64_t dgref_t2j3(const uint8_t *blob, const uint8_t *side, uint32_t root, const uint8_t *thrift, size_t n,
                    uint64_t opts, uint8_t *out, size_t cap, size_t *out_len, uint64_t *aux, const uint8_t *ans,
                    uint32_t n_ans)
{
    T2J c;
    t2j_init(&c, blob, side, opts);
    uint32_t seen = 0;
    c.opts = opts;
    c.aux = aux;
    c.ans = ans;
    c.n_ans = n_ans;
    c.seen = &seen;
    JBuf o = {(char *)malloc(256), 0, 256};
    uint64_t e = t2j_do(&c, root, thrift, n, &o);
    const int keep = !e || (e & 0xFF) == DG_T2J_E_EXCEPTION || (e & 0xFF) == DG_T2J_E_CALLBACK;
    *out_len = keep ? o.len : 0;
    if (keep && o.len <= cap)
        memcpy(out, o.b, o.len);
    free(o.b);
    return e;
}

/* ---- timed batch driver for bench.py's t2j cpu_baseline ----
 * Same shape as dgref_j2t_timed: pinned threads, byte-balanced contiguous
 * shards, one untimed pass then `reps` timed ones between barriers; each
 * message converted into a per-thread reused buffer and copied into its
 * output slot (Do's copy, conv/t2j/conv.go:67-70). */
typedef struct {
    T2J c;
    uint32_t root;
    const uint8_t *src;
    const uint64_t *in_off;
    uint64_t lo, hi;
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t *out_len;
    uint64_t *ret;
    int cpu, tid, reps;
    pthread_barrier_t *bar;
    double *best;
} T2JJob;

static void *run_t2j_timed(void *arg)
{
    T2JJob *t = (T2JJob *)arg;
    if (t->cpu >= 0) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(t->cpu, &cs);
        pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
    }
    JBuf o = {(char *)malloc(1 << 16), 0, 1 << 16};
    double t0 = 0;
    for (int rep = -1; rep < t->reps; rep++) {
        pthread_barrier_wait(t->bar);
        if (t->tid == 0)
            t0 = now_s();
        for (uint64_t i = t->lo; i < t->hi; i++) {
            uint64_t e = t2j_do(&t->c, t->root, t->src + t->in_off[i], t->in_off[i + 1] - t->in_off[i], &o);
            uint64_t cap = t->out_off[i + 1] - t->out_off[i];
            t->ret[i] = e;
            t->out_len[i] = e ? 0 : (uint32_t)o.len;
            if (!e && o.len <= cap)
                memcpy(t->out + t->out_off[i], o.b, o.len);
        }
        pthread_barrier_wait(t->bar);
        if (t->tid == 0 && rep >= 0) {
            double dt = now_s() - t0;
            if (t->best[0] < 0 || dt < t->best[0])
                t->best[0] = dt;
            t->best[1 + rep] = dt;
        }
    }
    free(o.b);
    return NULL;
}

int dgref_t2j_timed(const uint8_t *blob, const uint8_t *side, uint32_t root, const uint8_t *src,
                    const uint64_t *in_off, uint64_t n, uint64_t opts, uint8_t *out, const uint64_t *out_off,
                    uint32_t *out_len, uint64_t *ret, int nthreads, const int *cpus, int reps, double *best_s)
{
    if (nthreads < 1 || reps < 1 || !best_s)
        return -1;
    T2JJob *tj = (T2JJob *)calloc(nthreads, sizeof(T2JJob));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    best_s[0] = -1;
    uint64_t total = in_off[n] - in_off[0];
    uint64_t lo = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t target = in_off[0] + total * (uint64_t)(t + 1) / nthreads;
        uint64_t hi = lo;
        while (hi < n && (t == nthreads - 1 || in_off[hi] < target))
            hi++;
        t2j_init(&tj[t].c, blob, side, opts);
        tj[t].root = root;
        tj[t].src = src;
        tj[t].in_off = in_off;
        tj[t].lo = lo;
        tj[t].hi = hi;
        tj[t].out = out;
        tj[t].out_off = out_off;
        tj[t].out_len = out_len;
        tj[t].ret = ret;
        tj[t].cpu = cpus ? cpus[t] : -1;
        tj[t].tid = t;
        tj[t].reps = reps;
        tj[t].bar = &bar;
        tj[t].best = best_s;
        lo = hi;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, run_t2j_timed, &tj[t]);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    free(tj);
    free(th);
    return 0;
}

/* The reference's UTF-8 validator, utf8_validate (native/utf8.c:183-212):
 * -1 if s[0, n) is valid UTF-8, else the offset of the first invalid
 * sequence. Not on the reference's j2t path; it pins the verdicts of the
 * opt-in DG_F_VALIDATE_UTF8 extension (tests/test_oracle.py,
 * tests/test_gpu_parity.py). */
long dgref_utf8_validate(const uint8_t *s, size_t n) { return (long)utf8_validate((const char *)s, (ssize_t)n); }
