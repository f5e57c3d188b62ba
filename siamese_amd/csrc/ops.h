// ops.h -- descriptors handed from the host control plane to the MI355X
// kernels.  Plain POD, shared verbatim by host C++ and HIP device code.
//
// Execution model (see DESIGN.md "Device program"):
//   * Every codec instance (one encoder or one decoder) owns an ordered list
//     of ops.  Ops of different instances are independent.
//   * All symbol arithmetic is byte-column local (byte i of every operand
//     only meets byte i of the others), so the executor runs each instance's
//     op list once per 1 KiB byte tile, in parallel over (instance, tile),
//     with no synchronisation between workgroups.
//   * The triangular solve of a decode needs the recovered length prefix
//     (bytes 0..3) before it can truncate later rows, so it is a separate
//     pair of launches (solve_prefix, solve_main) between executor segments.
#pragma once

#include <cstdint>

namespace sgpu {

/// One source of a linear combination: contributes coeff * src[0, len).
struct GfTerm
{
    uint64_t src;     // device address
    uint32_t len;     // bytes read from src (host guarantees len <= op.n)
    uint8_t coeff;    // GF(256) multiplier; 1 = plain XOR
    uint8_t acc;      // accumulator 0 (direct) or 1 (multiplied by op.mix)
    uint16_t pad;
};

enum GfOpKind : uint32_t
{
    OP_LINCOMB = 1,   // dst[0,n) = keep(dst,valid) ^ acc0 ^ mix*acc1
    OP_LITERAL = 2,   // dst[n, n+valid) = literal bytes (<= 8)
    OP_ROWS = 3,      // a batch of Siamese rows sharing one set of lane sums
    OP_ROW = 4,       // one row of the enclosing OP_ROWS batch (stream item)
};

/// One op.  For OP_LINCOMB:
///   for i < n:  dst[i] = (i < valid ? dst[i] : 0) ^ sum_{acc0 terms} c*src[i]
///                        ^ mix * sum_{acc1 terms} c*src[i]
///   bytes of dst at i >= n are left untouched.
/// For OP_LITERAL: writes `valid` (<= 8) bytes taken from `lit` at dst + n.
struct GfOp
{
    uint64_t dst;
    uint32_t n;
    uint32_t valid;
    uint32_t kind;
    uint32_t mix;
    union {
        struct {
            uint32_t termBegin;
            uint32_t termCount;
        };
        uint8_t lit[8];
    };
};
static_assert(sizeof(GfOp) == 32, "GfOp layout");
static_assert(sizeof(GfTerm) == 16, "GfTerm layout");

/// On the device a segment is one instruction stream of 16-byte words: each
/// op is its GfOp (2 words) followed, for OP_LINCOMB, by its termCount
/// GfTerm words (termBegin is unused there).  A workgroup streams through it
/// front to back, so one coalesced prefetch brings an op and its term list.
constexpr unsigned kOpWords = sizeof(GfOp) / 16;

/// OP_ROWS (Siamese rows, reference SiameseEncoder.cpp:1046-1144 and the
/// decoder's elimination SiameseDecoder.cpp:937-1038).  Stream layout:
///   GfOp header   kind=OP_ROWS, n = rows K, valid = table entries T,
///                 mix = lane-sum entries S, termCount = T
///   T words       the source table as GfTerm {src, len}: the S lane sums
///                 of the batch first, then every distinct symbol an LDPC
///                 pair of some row picked
///   K row items, each RowHeader (3 words) + pick words:
///     dst[0,n) = keep(dst,valid) ^ acc0 ^ mix * acc1 over the row's picks
///     (uint16 table index | acc << 15, eight per word: the sums its opcode
///     selects, then its LDPC pairs), then `litLen` literal bytes (the
///     recovery footer) at dst+n.
/// All rows of a batch share one table, so the host sends 2 bytes per
/// source instead of a 16-byte term, and the sums stay hot on the device.
struct RowHeader
{
    uint64_t dst;
    uint32_t n;
    uint32_t valid;
    uint32_t kindPicks;   // OP_ROW | npicks << 8
    uint32_t mix;         // RX multiplier of acc1 | litLen << 8
    uint32_t reserved[2];
    uint8_t lit[8];       // literal bytes written at dst + n
    uint32_t pad[2];
};
static_assert(sizeof(RowHeader) == 48, "RowHeader layout");
constexpr unsigned kRowWords = sizeof(RowHeader) / 16;
constexpr unsigned kPicksPerWord = 8;
constexpr unsigned kMaxRowsTable = 0x7fff;   // table indices fit 15 bits

inline uint32_t op_words(const GfOp& op)
{
    // (an OP_ROWS header's words cover its table; its rows follow as items)
    return kOpWords + ((op.kind == OP_LINCOMB || op.kind == OP_ROWS) ? op.termCount : 0);
}

/// Executor work item: one (instance segment, byte tile).
struct ExecItem
{
    uint32_t streamBegin;  // first 16-byte word of the segment's stream
    uint32_t streamWords;  // words in the segment's stream
    uint32_t opCount;
    uint32_t tileBase;     // first byte of this tile
};

/// Triangular solve of one decode (reference SiameseDecoder.cpp:1065-1238).
/// Rows are listed in pivot order; coef is an m x m byte matrix with
/// coef[j*m + i] = RecoveryMatrix[Pivots[j]][i].
struct SolveDesc
{
    uint32_t m;
    uint32_t rowBegin;   // index into SolveRow array
    uint64_t coefOffset; // byte offset into coefficient array
    uint32_t result;     // index into the uint32 result array (m+1 words)
    uint32_t maxBytes;   // max finalBytes over rows (tile count)
};

struct SolveRow
{
    uint64_t buf;        // recovery buffer (becomes the recovered original)
    uint32_t initBytes;  // Bytes before MultiplyLowerTriangle
    uint32_t lowerLen;   // Bytes when this row is the source of the lower step
    uint32_t finalBytes; // Bytes after MultiplyLowerTriangle
    uint32_t pad;
};

/// Result word layout for each recovered row: (headerBytes << 29) | length,
/// or 0 if the prefix failed validation.  Word 0 holds the number of rows
/// recovered before the first invalid one (== m when all are valid), counting
/// from the right-most column as the reference does.
constexpr uint32_t kSolveLengthMask = 0x1fffffffu;

/// Solve work item: one (solve, byte tile).
struct SolveItem
{
    uint32_t solve;
    uint32_t tileBase;
};

/// Ingest of one symbol into a FRESH device buffer (never referenced by any
/// op of the same flush before this point), so ingest can run as the first
/// launch of a flush:  dst[0,hdrLen) = hdr,  dst[hdrLen, hdrLen+bytes) = src,
/// and dst[total, align16(total)) = 0 (whole 16-byte lanes are stored; dst is
/// 16-byte aligned with capacity >= align16(total)).
struct IngestDesc
{
    uint64_t dst;
    uint64_t src;
    uint32_t bytes;
    uint32_t hdrLen;
    uint8_t hdr[8];
};

constexpr unsigned kTileBytes = 1024;   // 64 lanes x 16 bytes

} // namespace sgpu
