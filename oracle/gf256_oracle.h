/*
    oracle/gf256_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the
    product).  A plain-C restatement of the reference's GF(2^8) layer and code
    definition, used by tests/ to pin known answers.  Full-codec parity is
    pinned by the unmodified reference built into oracle/_ref/libsiamese_ref.so.

    Parity status: PINNED.  Every function below is checked by
    tests/test_oracle.py against the reference's own self-test vectors
    (gf256.cpp:84-189), its serializer tests (tests/test_serializers.cpp) and
    outputs of the compiled reference (SURVEY.md section 8c known answers).
*/
#ifndef GF256_ORACLE_H
#define GF256_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gf256.cpp:357-464 -- tables over polynomial 0x14D */
int orc_init(void);
uint8_t orc_mul(uint8_t x, uint8_t y);
uint8_t orc_div(uint8_t x, uint8_t y);
uint8_t orc_inv(uint8_t x);
uint8_t orc_sqr(uint8_t x);
uint8_t orc_exp(unsigned i);
unsigned orc_log(uint8_t x);
unsigned orc_poly(void);

/* gf256.cpp:653-1495 -- bulk ops (scalar) */
void orc_add_mem(uint8_t* x, const uint8_t* y, int bytes);              /* x ^= y      */
void orc_mul_mem(uint8_t* z, const uint8_t* x, uint8_t y, int bytes);   /* z = x*y     */
void orc_muladd_mem(uint8_t* z, uint8_t y, const uint8_t* x, int bytes);/* z ^= x*y    */

/* SiameseCommon.h:89-218 */
uint8_t orc_column_value(unsigned column);
uint8_t orc_row_value(unsigned row);
unsigned orc_row_opcode(unsigned lane, unsigned row);
uint8_t orc_cauchy_element(unsigned row, unsigned column);
uint32_t orc_int32_hash(uint32_t key);

/* SiameseTools.h:80-102 -- writes `count` outputs after Seed(y, x) */
void orc_pcg(uint64_t y, uint64_t x, uint32_t* out, unsigned count);

/* SiameseSerializers.h:566-627, 736-800 */
unsigned orc_write_length(unsigned length, uint8_t* out);
int orc_read_length(const uint8_t* in, unsigned avail, unsigned* length);
unsigned orc_write_footer(unsigned row, unsigned columnStart, unsigned sumCount,
                          unsigned ldpcCount, uint8_t* out);
int orc_read_footer(const uint8_t* data, unsigned bytes, unsigned* row, unsigned* columnStart,
                    unsigned* sumCount, unsigned* ldpcCount);

/* SiameseSerializers.h:854-994 -- NACK loss range */
unsigned orc_write_nack(unsigned relativeStart, unsigned lossCountM1, uint8_t* out);
int orc_read_nack(const uint8_t* in, unsigned avail, unsigned* relativeStart,
                  unsigned* lossCountM1);

/*
    SiameseEncoder.cpp:1046-1254 -- one Siamese recovery row over a window
    whose running sums are built from scratch (the encoder state right after
    ResetSums(0) and `count` Add() calls with ColumnStart 0).  symbols[i] holds
    `len[i]` bytes (length prefix included); `out` receives recoveryBytes
    (= max len) bytes.  Restated for tests of the device row math.
*/
void orc_siamese_row(const uint8_t* const* symbols, const unsigned* len, unsigned count,
                     unsigned row, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif
