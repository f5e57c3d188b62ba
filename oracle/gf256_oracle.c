/*
    oracle/gf256_oracle.c -- TEST INFRASTRUCTURE ONLY.  See gf256_oracle.h.
    Scalar, table-driven restatement; each function cites the reference
    definition it follows.  Nothing here is linked into the product library.
*/
#include "gf256_oracle.h"

#include <stdlib.h>
#include <string.h>

static uint8_t EXP[1024];
static uint16_t LOG[256];
static uint8_t MUL[256][256];
static uint8_t DIV[256][256];
static uint8_t INV[256];
static uint8_t SQR[256];
static unsigned POLY;
static int READY;

int orc_init(void)
{
    if (READY)
        return 0;
    /* gf256.cpp:357-372: GF256_GEN_POLY[3] = 0xa6 -> (0xa6 << 1) | 1 */
    POLY = (0xa6u << 1) | 1u;
    /* gf256.cpp:379-403: log[0] = 512, exp doubled, exp[510] = 1, rest 0 */
    LOG[0] = 512;
    EXP[0] = 1;
    for (unsigned j = 1; j < 255; ++j) {
        unsigned next = (unsigned)EXP[j - 1] * 2;
        if (next >= 256)
            next ^= POLY;
        EXP[j] = (uint8_t)next;
        LOG[EXP[j]] = (uint16_t)j;
    }
    EXP[255] = EXP[0];
    LOG[EXP[255]] = 255;
    for (unsigned j = 256; j < 2 * 255; ++j)
        EXP[j] = EXP[j % 255];
    EXP[2 * 255] = 1;
    for (unsigned j = 2 * 255 + 1; j < 4 * 255; ++j)
        EXP[j] = 0;
    /* gf256.cpp:410-442 */
    for (unsigned y = 0; y < 256; ++y) {
        for (unsigned x = 0; x < 256; ++x) {
            if (x == 0 || y == 0) {
                MUL[y][x] = 0;
                DIV[y][x] = 0;
                continue;
            }
            const unsigned ly = (uint8_t)LOG[y];
            MUL[y][x] = EXP[LOG[x] + ly];
            DIV[y][x] = EXP[LOG[x] + 255 - ly];
        }
    }
    /* gf256.cpp:449-464 */
    for (unsigned x = 0; x < 256; ++x) {
        INV[x] = DIV[x][1];
        SQR[x] = MUL[x][x];
    }
    READY = 1;
    return 0;
}

uint8_t orc_mul(uint8_t x, uint8_t y) { return MUL[y][x]; }
uint8_t orc_div(uint8_t x, uint8_t y) { return DIV[y][x]; }
uint8_t orc_inv(uint8_t x) { return INV[x]; }
uint8_t orc_sqr(uint8_t x) { return SQR[x]; }
uint8_t orc_exp(unsigned i) { return EXP[i & 1023]; }
unsigned orc_log(uint8_t x) { return LOG[x]; }
unsigned orc_poly(void) { return POLY; }

void orc_add_mem(uint8_t* x, const uint8_t* y, int bytes)
{
    for (int i = 0; i < bytes; ++i)
        x[i] ^= y[i];
}

void orc_mul_mem(uint8_t* z, const uint8_t* x, uint8_t y, int bytes)
{
    for (int i = 0; i < bytes; ++i)
        z[i] = MUL[y][x[i]];
}

void orc_muladd_mem(uint8_t* z, uint8_t y, const uint8_t* x, int bytes)
{
    for (int i = 0; i < bytes; ++i)
        z[i] ^= MUL[y][x[i]];
}

/* SiameseCommon.h:89-98 */
uint8_t orc_column_value(unsigned column) { return (uint8_t)(3 + (column * 199) % 253); }
uint8_t orc_row_value(unsigned row) { return (uint8_t)(1 + (row + 1) % 255); }

/* SiameseCommon.h:150-159 */
uint32_t orc_int32_hash(uint32_t key)
{
    key += ~(key << 15);
    key ^= (key >> 10);
    key += (key << 3);
    key ^= (key >> 6);
    key += ~(key << 11);
    key ^= (key >> 16);
    return key;
}

/* SiameseCommon.h:162-174 */
unsigned orc_row_opcode(unsigned lane, unsigned row)
{
    const uint32_t op = orc_int32_hash(lane + (row + 3) * 8) & 63;
    return op == 0 ? 16 : op;
}

/* SiameseCommon.h:212-218 */
uint8_t orc_cauchy_element(unsigned row, unsigned column)
{
    return INV[(uint8_t)((row + 64) ^ column)];
}

/* SiameseTools.h:80-102 */
typedef struct
{
    uint64_t state, inc;
} Pcg;

static uint32_t pcg_next(Pcg* p)
{
    const uint64_t old = p->state;
    p->state = old * 6364136223846793005ULL + p->inc;
    const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    const uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((uint32_t)(-(int32_t)rot) & 31));
}

static void pcg_seed(Pcg* p, uint64_t y, uint64_t x)
{
    p->state = 0;
    p->inc = (y << 1u) | 1u;
    pcg_next(p);
    p->state += x;
    pcg_next(p);
}

void orc_pcg(uint64_t y, uint64_t x, uint32_t* out, unsigned count)
{
    Pcg p;
    pcg_seed(&p, y, x);
    for (unsigned i = 0; i < count; ++i)
        out[i] = pcg_next(&p);
}

/* SiameseSerializers.h:566-593 */
unsigned orc_write_length(unsigned length, uint8_t* out)
{
    if (length <= 0x7f) {
        out[0] = (uint8_t)length;
        return 1;
    }
    if (length <= 0x3fff) {
        out[0] = (uint8_t)(0x80 | (length >> 8));
        out[1] = (uint8_t)length;
        return 2;
    }
    if (length <= 0x1fffff) {
        out[0] = (uint8_t)(0xC0 | (length >> 16));
        out[1] = (uint8_t)(length >> 8);
        out[2] = (uint8_t)length;
        return 3;
    }
    out[0] = (uint8_t)(0xE0 | (length >> 24));
    out[1] = (uint8_t)(length >> 16);
    out[2] = (uint8_t)(length >> 8);
    out[3] = (uint8_t)length;
    return 4;
}

/* SiameseSerializers.h:596-627 */
int orc_read_length(const uint8_t* in, unsigned avail, unsigned* length)
{
    if (!in || avail < 1)
        return -1;
    const int n = in[0] >> 6;
    if (n <= 1) {
        *length = in[0];
        return 1;
    }
    if (n == 2) {
        if (avail < 2)
            return -1;
        *length = (((unsigned)in[0] << 8) | in[1]) & 0x3fff;
        return 2;
    }
    if ((in[0] & 0xE0) == 0xC0) {
        if (avail < 3)
            return -1;
        *length = (((unsigned)in[0] << 16) | ((unsigned)in[1] << 8) | in[2]) & 0x1fffff;
        return 3;
    }
    if (avail < 4)
        return -1;
    *length = (((unsigned)in[0] << 24) | ((unsigned)in[1] << 16) | ((unsigned)in[2] << 8) | in[3]) &
              0x1fffffff;
    return 4;
}

/* SiameseSerializers.h:383-400 (PacketNum footer) and :510-526 (count footer) */
static unsigned put_num(unsigned v, uint8_t* b)
{
    if (v <= 0x7f) {
        b[0] = (uint8_t)v;
        return 1;
    }
    if (v <= 0x3fff) {
        b[0] = (uint8_t)v;
        b[1] = (uint8_t)(0x80 | (v >> 8));
        return 2;
    }
    b[0] = (uint8_t)v;
    b[1] = (uint8_t)(v >> 8);
    b[2] = (uint8_t)(0xC0 | (v >> 16));
    return 3;
}

static unsigned put_count(unsigned v, uint8_t* b)
{
    if (v <= 127) {
        b[0] = (uint8_t)v;
        return 1;
    }
    b[0] = (uint8_t)v;
    b[1] = (uint8_t)(0x80 | (v >> 8));
    return 2;
}

/* SiameseSerializers.h:736-754 */
unsigned orc_write_footer(unsigned row, unsigned columnStart, unsigned sumCount, unsigned ldpcCount,
                          uint8_t* out)
{
    unsigned n = 0;
    if (sumCount > 1) {
        out[n++] = (uint8_t)row;
        n += put_count(ldpcCount, out + n);
    }
    n += put_num(columnStart, out + n);
    n += put_count(sumCount - 1, out + n);
    return n;
}

static int get_count(const uint8_t* b, unsigned avail, unsigned* v)
{
    if (avail < 1)
        return -1;
    b += avail - 1;
    if (!(b[0] & 0x80)) {
        *v = b[0];
        return 1;
    }
    if (avail < 2)
        return -1;
    *v = (((unsigned)b[0] << 8) | b[-1]) & 0x7fff;
    return 2;
}

static int get_num(const uint8_t* b, int avail, unsigned* v)
{
    if (!b || avail < 1)
        return -1;
    b += avail - 1;
    const int n = b[0] >> 6;
    if (n <= 1) {
        *v = b[0];
        return 1;
    }
    if (avail < n)
        return -1;
    if (n == 2)
        *v = (((unsigned)b[0] << 8) | b[-1]) & 0x3fff;
    else
        *v = (((unsigned)b[0] << 16) | ((unsigned)b[-1] << 8) | b[-2]) & 0x3fffff;
    return n;
}

/* SiameseSerializers.h:759-800 */
int orc_read_footer(const uint8_t* data, unsigned bytes, unsigned* row, unsigned* columnStart,
                    unsigned* sumCount, unsigned* ldpcCount)
{
    unsigned left = bytes;
    int w = get_count(data, left, sumCount);
    if (w < 0)
        return -1;
    left -= w;
    *sumCount += 1;
    w = get_num(data, (int)left, columnStart);
    if (w < 0)
        return -1;
    left -= w;
    if (*sumCount <= 1) {
        *ldpcCount = 1;
        *row = 0;
    } else {
        w = get_count(data, left, ldpcCount);
        if (w < 0)
            return -1;
        left -= w;
        if (*sumCount < *ldpcCount)
            return -1;
        if (left < 1)
            return -1;
        *row = data[--left];
    }
    return (int)(bytes - left);
}

/* SiameseSerializers.h:854-930 */
unsigned orc_write_nack(unsigned rs, unsigned lm1, uint8_t* b)
{
    unsigned b0 = (lm1 <= 2 ? lm1 : 3) | (rs << 3);
    unsigned n = 1;
    if (rs >= 32) {
        unsigned b1 = rs >> 5;
        if (rs >= (1u << 12)) {
            unsigned b2 = rs >> 12;
            if (rs >= (1u << 19)) {
                b[3] = (uint8_t)(rs >> 19);
                b2 |= 0x80;
                ++n;
            }
            b[2] = (uint8_t)b2;
            b1 |= 0x80;
            ++n;
        }
        b[1] = (uint8_t)b1;
        b0 |= 4;
        ++n;
    }
    b[0] = (uint8_t)b0;
    if (lm1 >= 3) {
        uint8_t* e = b + n;
        unsigned x = lm1 - 3, e1 = x;
        if (x >= 128) {
            unsigned e2 = x >> 7;
            if (x >= (1u << 14)) {
                e[2] = (uint8_t)(x >> 14);
                e2 |= 0x80;
                ++n;
            }
            e[1] = (uint8_t)e2;
            e1 |= 0x80;
            ++n;
        }
        e[0] = (uint8_t)e1;
        ++n;
    }
    return n;
}

/* SiameseSerializers.h:936-994 */
int orc_read_nack(const uint8_t* b, unsigned avail, unsigned* rs, unsigned* lm1)
{
    if (!b || avail < 7)
        return -1;
    unsigned loss = b[0] & 3, rel = b[0] >> 3, n = 1;
    if (b[0] & 4) {
        ++n;
        rel |= (b[1] & 0x7fu) << 5;
        if (b[1] & 0x80) {
            ++n;
            rel |= (b[2] & 0x7fu) << 12;
            if (b[2] & 0x80) {
                ++n;
                rel |= (unsigned)b[3] << 19;
            }
        }
    }
    if (loss == 3) {
        const uint8_t* e = b + n;
        loss += e[0] & 0x7f;
        if (e[0] & 0x80) {
            loss += (e[1] & 0x7fu) << 7;
            if (e[1] & 0x80) {
                loss += (unsigned)e[2] << 14;
                ++n;
            }
            ++n;
        }
        ++n;
    }
    *rs = rel;
    *lm1 = loss;
    return (int)n;
}

/* SiameseEncoder.cpp:359-418 (GetSum), :1046-1144 (dense + light columns),
   :1229-1233 (RX * product) for a window starting at column 0. */
void orc_siamese_row(const uint8_t* const* sym, const unsigned* len, unsigned count, unsigned row,
                     uint8_t* out)
{
    unsigned recoveryBytes = 0, laneLongest[8] = {0};
    for (unsigned e = 0; e < count; ++e) {
        if (len[e] > recoveryBytes)
            recoveryBytes = len[e];
        if (len[e] > laneLongest[e % 8])
            laneLongest[e % 8] = len[e];
    }
    uint8_t* sums[8][3];
    for (unsigned l = 0; l < 8; ++l)
        for (unsigned s = 0; s < 3; ++s) {
            sums[l][s] = (uint8_t*)calloc(laneLongest[l] + 1, 1);
            for (unsigned e = l; e < count; e += 8) {
                uint8_t cx = orc_column_value(e);
                if (s == 2)
                    cx = SQR[cx];
                if (s == 0)
                    orc_add_mem(sums[l][s], sym[e], (int)len[e]);
                else
                    orc_muladd_mem(sums[l][s], cx, sym[e], (int)len[e]);
            }
        }
    uint8_t* prod = (uint8_t*)calloc(recoveryBytes + 1, 1);
    memset(out, 0, recoveryBytes);
    for (unsigned l = 0; l < 8; ++l) {
        const unsigned op = orc_row_opcode(l, row);
        for (unsigned bit = 0; bit < 6; ++bit) {
            if (!(op & (1u << bit)) || laneLongest[l] == 0)
                continue;
            unsigned n = laneLongest[l] < recoveryBytes ? laneLongest[l] : recoveryBytes;
            orc_add_mem(bit < 3 ? out : prod, sums[l][bit % 3], (int)n);
        }
    }
    Pcg p;
    pcg_seed(&p, row, count);
    const unsigned pairs = (count + 15) / 16;
    for (unsigned i = 0; i < pairs; ++i) {
        const unsigned e1 = pcg_next(&p) % count;
        const unsigned e2 = pcg_next(&p) % count;
        orc_add_mem(out, sym[e1], (int)len[e1]);
        orc_add_mem(prod, sym[e2], (int)len[e2]);
    }
    orc_muladd_mem(out, orc_row_value(row), prod, (int)recoveryBytes);
    for (unsigned l = 0; l < 8; ++l)
        for (unsigned s = 0; s < 3; ++s)
            free(sums[l][s]);
    free(prod);
}
