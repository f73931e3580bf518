/*
 * fuzz_oracle.c — randomized/mutational driver for the CPU oracle, built
 * with AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile
 * `fuzz_asan`). TEST INFRASTRUCTURE: it checks the checker.
 *
 * It restates the reference's two cargo-fuzz targets over generated inputs
 * (no libFuzzer here; a seeded generator of valid messages and mutations of
 * them stands in for the corpus):
 *
 *   fuzz/fuzz_targets/parse_serialise.rs:5-12
 *     decode(data) == Ok(m)  =>  serialise(m) decodes again, to m.
 *   fuzz/fuzz_targets/bytes.rs:8-23
 *     Bytes decode Ok(m)  =>  slice decode Ok too and both re-serialise to
 *     the same bytes;  Bytes decode Err  =>  slice decode Err.
 *
 * Every input is copied into a heap block of exactly its length, so any
 * read past the end of a message (the bounds the reference's Cursor /
 * Bytes readers enforce) is an ASan report, and any signed overflow or
 * misaligned access is a UBSan abort.
 *
 * Usage: fuzz_oracle_asan [iterations] [seed]   (exit 0 = no violation)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "onc_oracle.h"

static uint64_t rng_state;

static uint64_t next_u64(void) {   /* splitmix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint32_t rnd(uint32_t n) { return n ? (uint32_t)(next_u64() % n) : 0; }

/* ------------------------------------------------------------------------ */
/* generator of valid messages (descriptor form), like the reference's       */
/* proptest strategies (rpc_message.rs:997-1124)                             */
/* ------------------------------------------------------------------------ */
typedef struct {
    onc_msg msg;
    onc_unix_params unix[2];
    uint8_t arena[2 * 260 + 2048];   /* auth bodies, names, payload */
    uint32_t used;
} gen_msg;

static uint32_t put_bytes(gen_msg* g, uint32_t len) {
    const uint32_t off = g->used;
    for (uint32_t i = 0; i < len; ++i) g->arena[off + i] = (uint8_t)next_u64();
    g->used += len;
    return off;
}

static void gen_auth(gen_msg* g, onc_auth* a, int slot) {
    const uint32_t k = rnd(4);
    if (k == ONC_KIND_UNIX) {
        onc_unix_params* u = &g->unix[slot];
        memset(u, 0, sizeof(*u));
        u->stamp = (uint32_t)next_u64();
        u->uid = (uint32_t)next_u64();
        u->gid = (uint32_t)next_u64();
        u->ngids = rnd(17);
        for (uint32_t i = 0; i < u->ngids; ++i) u->gids[i] = (uint32_t)next_u64();
        u->name_len = rnd(2) ? rnd(17) : rnd(200 - 12 - 4 * u->ngids + 1);   /* assoc <= 200 */
        u->name_off = put_bytes(g, u->name_len);
        a->id = ONC_AUTH_UNIX;
        a->kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, 0);
        a->ref = (uint64_t)slot;
        return;
    }
    const uint32_t len = rnd(3) ? rnd(33) : rnd(201);
    a->id = k == ONC_KIND_NONE ? ONC_AUTH_NONE : k == ONC_KIND_SHORT ? ONC_AUTH_SHORT : 3u + rnd(0xFFFFFFF0u);
    a->kind_len = ONC_AUTH_PACK(k, len);
    a->ref = put_bytes(g, len);
}

static void gen_message(gen_msg* g) {
    memset(g, 0, sizeof(*g));
    onc_msg* m = &g->msg;
    m->xid = (uint32_t)next_u64();
    const uint32_t t = rnd(4);
    if (t < 2) {
        m->msg_type = ONC_MSG_CALL;
        m->u.call.program = (uint32_t)next_u64();
        m->u.call.program_version = (uint32_t)next_u64();
        m->u.call.procedure = (uint32_t)next_u64();
        gen_auth(g, &m->cred, 0);
        gen_auth(g, &m->verf, 1);
        m->payload_len = rnd(2) ? rnd(64) : rnd(1026);
        m->payload_off = put_bytes(g, m->payload_len);
        return;
    }
    m->msg_type = ONC_MSG_REPLY;
    if (t == 2) {
        m->reply_stat = ONC_REPLY_ACCEPTED;
        gen_auth(g, &m->verf, 1);
        m->stat = (uint8_t)rnd(6);
        if (m->stat == ONC_ACCEPT_SUCCESS) {
            m->payload_len = rnd(300);
            m->payload_off = put_bytes(g, m->payload_len);
        } else if (m->stat == ONC_ACCEPT_PROG_MISMATCH) {
            m->u.mismatch.low = (uint32_t)next_u64();
            m->u.mismatch.high = (uint32_t)next_u64();
        }
        return;
    }
    m->reply_stat = ONC_REPLY_DENIED;
    m->stat = (uint8_t)rnd(2);
    if (m->stat == ONC_REJECT_RPC_MISMATCH) {
        m->u.mismatch.low = (uint32_t)next_u64();
        m->u.mismatch.high = (uint32_t)next_u64();
    } else {
        m->auth_stat = (uint8_t)rnd(8);
    }
}

/* ------------------------------------------------------------------------ */
/* mutations (the corrupted-record kinds of the GPU differential tests)      */
/* ------------------------------------------------------------------------ */
static void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

static uint64_t mutate(uint8_t* buf, uint64_t len, uint64_t cap) {
    const uint32_t op = rnd(7);
    if (op == 0 && len) {                                  /* flip a byte */
        buf[rnd((uint32_t)len)] ^= (uint8_t)(1 + rnd(255));
    } else if (op == 1 && len) {                           /* truncate */
        len = rnd((uint32_t)len);
    } else if (op == 2 && len + 16 <= cap) {               /* trailing bytes, header fixed up */
        const uint32_t k = 1 + rnd(12);
        for (uint32_t i = 0; i < k; ++i) buf[len + i] = (uint8_t)next_u64();
        len += k;
        if (len >= 4) put_be32(buf, (uint32_t)(len - 4) | 0x80000000u);
    } else if (op == 3 && len >= 4) {                      /* clear the last-fragment bit */
        buf[0] &= 0x7F;
    } else if (op == 4 && len >= 8) {                      /* small value into a header word */
        const uint32_t w = 1 + rnd((uint32_t)(len / 4 < 40 ? len / 4 - 1 : 39));
        put_be32(buf + 4 * w, rnd(300));
    } else if (op == 5 && len >= 8) {                      /* huge value into a header word */
        const uint32_t w = 1 + rnd((uint32_t)(len / 4 < 40 ? len / 4 - 1 : 39));
        put_be32(buf + 4 * w, 0xFFFFFF00u | rnd(256));
    } else if (len >= 4) {                                 /* random body, valid record mark */
        for (uint64_t i = 4; i < len; ++i) buf[i] = (uint8_t)next_u64();
        put_be32(buf, (uint32_t)(len - 4) | 0x80000000u);
    }
    return len;
}

/* ------------------------------------------------------------------------ */
/* the two fuzz invariants                                                   */
/* ------------------------------------------------------------------------ */
typedef struct {
    int32_t st;
    onc_msg msg;
    onc_unix_params unix[2];
} decoded;

static void dec(const uint8_t* data, uint64_t len, int mode, decoded* d) {
    uint32_t a0 = 0, a1 = 0;
    memset(d, 0, sizeof(*d));
    d->st = oracle_decode_message(data, data, len, mode, 0, &d->msg, d->unix, &a0, &a1);
}

/* serialise(m) of a decoded message (arenas = the buffer it borrows from),
 * into a heap block of exactly serialised_len bytes. */
static uint8_t* reserialise(const decoded* d, const uint8_t* data, uint64_t* out_len) {
    uint64_t written = 0, slen = 0;
    int32_t st = oracle_encode_message(&d->msg, d->unix, data, data, NULL, 0, &written, &slen);
    (void)st;
    uint8_t* out = (uint8_t*)malloc(slen ? slen : 1);
    st = oracle_encode_message(&d->msg, d->unix, data, data, out, slen, &written, &slen);
    if (st != ONC_OK || written != slen) {
        fprintf(stderr, "serialise of a decoded message failed: status %d written %llu of %llu\n", st,
                (unsigned long long)written, (unsigned long long)slen);
        exit(2);
    }
    *out_len = slen;
    return out;
}

static int same_unix(const decoded* a, const decoded* b, const onc_auth* x, int slot) {
    if ((x->kind_len >> 24) != ONC_KIND_UNIX) return 1;
    return memcmp(&a->unix[slot], &b->unix[slot], sizeof(onc_unix_params)) == 0;
}

static unsigned long long n_ok[2], n_err[2];

static void check(const uint8_t* src, uint64_t len) {
    uint8_t* data = (uint8_t*)malloc(len ? len : 1);   /* exactly len bytes: ASan bounds */
    memcpy(data, src, len);
    for (int mode = 0; mode < 2; ++mode) {
        decoded d;
        dec(data, len, mode, &d);
        if (d.st != ONC_OK) { ++n_err[mode]; continue; }
        ++n_ok[mode];
        /* parse_serialise.rs:5-12 */
        uint64_t l2 = 0;
        uint8_t* b2 = reserialise(&d, data, &l2);
        decoded d2;
        dec(b2, l2, mode, &d2);
        if (d2.st != ONC_OK || l2 != len || memcmp(&d.msg, &d2.msg, sizeof(onc_msg)) != 0 ||
            !same_unix(&d, &d2, &d.msg.cred, 0) || !same_unix(&d, &d2, &d.msg.verf, 1)) {
            fprintf(stderr, "parse_serialise violated (mode %d, len %llu, status %d)\n", mode,
                    (unsigned long long)len, d2.st);
            exit(1);
        }
        free(b2);
    }
    /* bytes.rs:8-23 */
    decoded db, ds;
    dec(data, len, ONC_DECODE_BYTES, &db);
    dec(data, len, ONC_DECODE_SLICE, &ds);
    if (db.st == ONC_OK) {
        if (ds.st != ONC_OK) {
            fprintf(stderr, "bytes Ok but slice Err %d (len %llu)\n", ds.st, (unsigned long long)len);
            exit(1);
        }
        uint64_t lb = 0, ls = 0;
        uint8_t* bb = reserialise(&db, data, &lb);
        uint8_t* bs = reserialise(&ds, data, &ls);
        if (lb != ls || memcmp(bb, bs, lb) != 0) {
            fprintf(stderr, "bytes / slice re-serialisations differ (len %llu)\n", (unsigned long long)len);
            exit(1);
        }
        free(bb);
        free(bs);
    } else if (ds.st == ONC_OK) {
        fprintf(stderr, "bytes Err %d but slice Ok (len %llu)\n", db.st, (unsigned long long)len);
        exit(1);
    }
    free(data);
}

int main(int argc, char** argv) {
    const unsigned long long iters = argc > 1 ? strtoull(argv[1], NULL, 10) : 100000ull;
    rng_state = argc > 2 ? strtoull(argv[2], NULL, 10) : 1ull;
    static gen_msg g;
    static uint8_t buf[8192];
    for (unsigned long long it = 0; it < iters; ++it) {
        gen_message(&g);
        uint64_t written = 0, slen = 0;
        const int32_t st = oracle_encode_message(&g.msg, g.unix, g.arena, g.arena, buf, sizeof(buf) - 64, &written,
                                                 &slen);
        if (st != ONC_OK) {
            fprintf(stderr, "generator produced an unencodable message: %d\n", st);
            return 2;
        }
        uint64_t len = written;
        check(buf, len);                                    /* the valid message */
        const uint32_t rounds = 1 + rnd(3);
        for (uint32_t r = 0; r < rounds; ++r) len = mutate(buf, len, sizeof(buf));
        check(buf, len);                                    /* a mutant */
        if ((it & 7) == 0) {                                /* short random buffers */
            const uint64_t k = rnd(64);
            for (uint64_t i = 0; i < k; ++i) buf[i] = (uint8_t)next_u64();
            if (k >= 4 && rnd(2)) put_be32(buf, (uint32_t)(k - 4) | 0x80000000u);
            check(buf, k);
        }
    }
    printf("fuzz_oracle: %llu iterations; slice ok %llu err %llu; bytes ok %llu err %llu\n", iters, n_ok[0], n_err[0],
           n_ok[1], n_err[1]);
    return 0;
}
