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
    OP_ROWS = 3,      // a batch of Siamese rows of one codec (sum updates, rows)
    OP_COPIES = 4,    // independent copies dst[0,len) = src[0,len)
    OP_LINCOMBS = 5,  // independent OP_LINCOMBs (+ footer literals), one per wave
};

/// One op.  For OP_LINCOMB:
///   for i < n:  dst[i] = (i < valid ? dst[i] : 0) ^ sum_{acc0 terms} c*src[i]
///                        ^ mix * sum_{acc1 terms} c*src[i]
///   bytes of dst in [n, align16(n)) become zero and bytes at and beyond
///   align16(n) are left untouched.  Every symbol buffer therefore reads as
///   zero between its length and the end of its last 16-byte lane (k_ingest
///   and the solve keep the same rule), which the executor relies on when it
///   reads a term of length len < n.
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
/// GfTerm words.  On the device termBegin is the op's gate (every kind but
/// OP_LITERAL): 0, or 1 + a result word; the op is skipped when that word is
/// zero (a chained device elimination that failed, GeDesc kGeChained).  A workgroup streams through it
/// front to back, so one coalesced prefetch brings an op and its term list.
constexpr unsigned kOpWords = sizeof(GfOp) / 16;

/// OP_ROWS: a batch of Siamese rows of one codec (reference
/// SiameseEncoder.cpp:1046-1144 and :359-418, the decoder's elimination
/// SiameseDecoder.cpp:937-1063 and :1680-1739).  Everything symbol-sized is
/// expanded on the device: the lane-sum updates generate their own terms and
/// coefficients CX(column) / CX(column)^2 from a snapshot of the codec's
/// window, and each row generates its LDPC pair picks from PCG(row, n).  The
/// host sends O(1) words per row instead of a term per source.
///
/// Stream layout after the GfOp header (kind = OP_ROWS, n = rows R,
/// valid = window entries E, mix = sum updates U, termCount = block words,
/// dst low word = stageLo: the first window element the batch reads, where
/// the executor's LDS stage of the window starts; dst high word = Rv: the
/// rows [0, Rv) that may read versioned sums, kVersionRows at most, 0 when no
/// update of the batch joined after a row read its sum):
///   24 words   WinEntry of the lane sums as the rows read them (lane*3 + s)
///   E words    WinEntry of window elements [base, base+E): an absent
///              (lost) element has len 0 and contributes nothing
///   U words    SumUpdate, run before any row of the batch (no row of the
///              batch reads a sum updated in it before the update; ops.h
///              invariant kept by Program)
///   R*3 words  RowItem
struct WinEntry
{
    uint64_t src;
    uint32_t len;
    uint32_t column;     // packet number (selects CX for sum updates)
};

/// dst[0,n) = keep(dst,valid) ^ sum over elements e = from, from+8, ... < to
/// of coeff(e) * window[e], coeff = 1, CX(column) or CX(column)^2 (s = 0..2).
struct SumUpdate
{
    uint32_t dstLo, dstHi;
    uint32_t n;
    uint32_t valid : 30;
    uint32_t s : 2;
    uint32_t from;
    uint32_t to;
    uint32_t sum;        // which of the 24 lane sums the rows read (lane*3+s) dst is
    uint32_t pad;
};

/// One Siamese row: dst[0,n) = keep(dst,valid) ^ acc0 ^ mix*acc1 where
///   acc0 = sums selected by mask0 (bit lane*3+s) ^ window[ldpcOff + PCG_2i % ldpcN]
///   acc1 = sums selected by mask1              ^ window[ldpcOff + PCG_2i+1 % ldpcN]
/// over i < ceil(ldpcN/16) pairs of PCG.Seed(row, ldpcN) draws, then litLen
/// footer bytes at dst + n.
///
/// A row reads each sum as it stood when the row was made: the batch's sum
/// updates are incremental (each extends its sum over later window elements,
/// SumUpdate), so sum k as row r reads it is the sum after every update of
/// the batch with the contributions of the update's elements at or past the
/// row's `cutoff` (batch-relative element index) taken back out.  Rows made
/// one after another in a streaming encoder (each folding the originals
/// added since the previous one into the sums it reads) then share one batch
/// instead of a batch each.  A batch with such joins (Program::rows_update)
/// holds at most kVersionRows rows, and only short joins: the executor
/// computes the corrections of each (row, lane) pair in parallel.
constexpr unsigned kVersionRows = 16;
constexpr unsigned kVersionMaxSpan = 32;   // window elements one joining update may add
struct RowItem
{
    uint64_t dst;
    uint32_t n;
    uint32_t valid;
    uint32_t mask0;      // bits 0..23; bits 24..30: litLen; bit 31: kRowWide
    uint32_t mask1;      // bits 0..23; bits 24..31: mix (RX)
    uint32_t row;
    uint32_t ldpcN;
    uint32_t ldpcOff;
    uint32_t cutoff;     // sums as of window elements < cutoff (batch-relative)
    uint8_t lit[8];
};
/// RowItem.mask0 bit 31: a wide row whose LDPC sums k_ldpc computed
/// (LdpcItem): ldpcN = 0, and window entries ldpcOff / ldpcOff + 1 hold L0 /
/// L1, added to acc0 / acc1 as two draws would be.
constexpr uint32_t kRowWide = 1u << 31;
inline constexpr uint32_t row_lit_len(uint32_t mask0) { return (mask0 >> 24) & 0x7fu; }
static_assert(sizeof(WinEntry) == 16, "WinEntry layout");
static_assert(sizeof(SumUpdate) == 32, "SumUpdate layout");
static_assert(sizeof(RowItem) == 48, "RowItem layout");
constexpr unsigned kRowSums = 24;                       // kLanes * kSums
constexpr unsigned kUpdateWords = sizeof(SumUpdate) / 16;
constexpr unsigned kRowWords = sizeof(RowItem) / 16;

/// Wide rows (ldpcN >= kLdpcSplitMin): the O(window) LDPC part of a row is
/// too much for the one workgroup per tile that runs the codec's op list, so
/// k_ldpc computes it first, spread over the whole chip: item k covers pairs
/// [pair0, pair1) of PCG.Seed(row, N) on one 1 KiB tile and XORs
///   L0 = sum of the even draws' window elements  into dst[0, n)
///   L1 = sum of the odd draws' window elements   into dst[span, span + n)
/// (a zeroed scratch area; items of one row meet by atomic XOR).  The row in
/// the OP_ROWS block then carries kRowWide, ldpcN = 0 and ldpcOff = the
/// window index of two entries appended to the batch's window that name L0
/// and L1, and adds them to acc0 and acc1 like two draws.  The same bytes
/// meet in a different order, which GF(2^8) addition (XOR) does not see.
struct LdpcItem
{
    uint64_t win;        // device address of the batch's window entry 0 (WinEntry[])
    uint64_t dst;        // L0 at dst, L1 at dst + span
    uint32_t span;
    uint32_t n;          // row bytes
    uint32_t row;
    uint32_t N;          // PCG.Seed(row, N); element = off + draw % N
    uint32_t off;
    uint32_t tileBase;
    uint32_t pair0, pair1;
};
static_assert(sizeof(LdpcItem) == 48, "LdpcItem layout");
constexpr uint32_t kLdpcSplitMin = 512;      // ldpcN from which a row's picks go to k_ldpc
#ifndef SGPU_LDPC_PAIRS
#define SGPU_LDPC_PAIRS 64
#endif
constexpr uint32_t kLdpcTileBytes = 1024;    // k_ldpc tile: 64 lanes x 16 bytes
/// Pairs per k_ldpc item for a row of `bytes`: rows of large symbols (C5:
/// 64 tiles each) take SGPU_LDPC_PAIRS, which halves their atomics and item
/// count (C5 66-69 ms/run vs 68-81 with 32); rows of small symbols keep 32,
/// so their few tiles still spread over enough workgroups (C3: k_ldpc 10.3
/// vs 13.1 us per launch with 64).  profiles/r3g_ldpc_item_ab.txt, r3h traces.
constexpr uint32_t ldpc_pairs_per_item(uint32_t bytes)
{
    return bytes >= 16 * kLdpcTileBytes ? SGPU_LDPC_PAIRS : 32u;
}

/// OP_COPIES: n independent copies (the decoder taking in recovery packets,
/// reference SiameseDecoder.cpp:437), one CopyItem word pair each after the
/// GfOp header (termCount = 2n).  dst[0,len) = src[0,len) with the zero tail
/// of every write; copies of one batch never overlap, so the executor deals
/// them to its waves without barriers.
struct CopyItem
{
    uint64_t dst;
    uint64_t src;
    uint32_t len;
    uint32_t pad[3];
};
static_assert(sizeof(CopyItem) == 32, "CopyItem layout");
constexpr unsigned kCopyWords = sizeof(CopyItem) / 16;

/// OP_LINCOMBS: n mutually independent linear combinations (no item reads or
/// writes bytes another item of the batch writes), each optionally followed
/// by a literal (a recovery packet's footer) on its own dst.  After the GfOp
/// header (termCount = the block's words): n LcItem (3 words each), then the
/// items' GfTerm words; termStart is an item's first term word within the
/// block.  The executor gives each wave whole items, so a run of small
/// combinations (Cauchy / parity rows of a short window, reference
/// SiameseEncoder.cpp:1334-1441, and the decoder's elimination of received
/// originals from each recovery packet, SiameseDecoder.cpp:812-1063) costs
/// one memory round trip and one barrier instead of one per combination.
struct LcItem
{
    uint64_t dst;
    uint32_t n, valid;           // as OP_LINCOMB
    uint32_t termStart, termCount;
    uint32_t mixLit;             // mix | litLen << 8
    uint32_t litOffset;          // literal at dst + litOffset (litLen <= 8)
    uint8_t lit[8];
    uint32_t pad[2];
};
static_assert(sizeof(LcItem) == 48, "LcItem layout");
constexpr unsigned kLcWords = sizeof(LcItem) / 16;
constexpr unsigned kLcMaxTerms = 64;    // larger combinations keep all waves on one op
constexpr unsigned kLcMaxItems = 256;

/// PCG-XSH-RR as the reference seeds it (SiameseTools.h:80-102).
constexpr uint64_t kPcgMul = 6364136223846793005ULL;

inline uint32_t op_words(const GfOp& op)
{
    // (an OP_ROWS header's termCount is its whole block in words)
    return kOpWords +
           ((op.kind == OP_LINCOMB || op.kind == OP_ROWS || op.kind == OP_COPIES || op.kind == OP_LINCOMBS)
                ? op.termCount
                : 0);
}

/// Executor work item: one (instance segment, byte tile).
struct ExecItem
{
    uint32_t streamBegin;  // first 16-byte word of the segment's stream
    uint32_t streamWords;  // words in the segment's stream
    uint32_t opCount;
    uint32_t tiles;        // exec_tiles(first 256-byte tile, tile count): the workgroup runs
                           // the op list over each tile (op by op, every tile in turn)
};
/// ExecItem.tiles: the first tile in the low 24 bits (16M tiles of 256 B:
/// 4 GiB, past SIAMESE_MAX_PACKET_BYTES), the run's tile count (1..255) in
/// the high 8.
constexpr uint32_t kExecRunMax = 255;
constexpr uint32_t kExecFirstTileMask = 0xffffffu;
constexpr uint32_t exec_tiles(uint32_t firstTile, uint32_t count) { return firstTile | count << 24; }
constexpr uint32_t exec_first_tile(uint32_t tiles) { return tiles & kExecFirstTileMask; }
constexpr uint32_t exec_tile_count(uint32_t tiles) { return tiles >> 24; }

/// Triangular solve of one decode (reference SiameseDecoder.cpp:1065-1238).
/// Rows are listed in pivot order; coef is an m x m byte matrix with
/// coef[j*m + i] = RecoveryMatrix[Pivots[j]][i].
struct SolveDesc
{
    uint32_t m;
    uint32_t rowBegin;   // index into SolveRow array
    uint64_t coefOffset; // byte offset into coefficient array
    uint32_t result;     // index into the uint32 result array (m+2 words:
                         // [0] rows recovered, [1..m] lengths, [m+1] set
                         // when a product solve's rows have non-zero bytes
                         // past their recovered lengths)
    uint32_t maxBytes;   // max finalBytes over rows (tile count)
    uint64_t head;       // m x 16 bytes: each row's first 16 bytes as the solve
                         // starts (copied by the segment before it), so every
                         // tile can solve the length prefixes while tile 0
                         // overwrites the rows
    uint64_t tinv;       // device scratch of solve_t_bytes(m) for the solve's
                         // inverse T (product solves; 0: none)
    uint64_t xout;       // device scratch of solve_x_bytes(m, maxBytes): the
                         // product solves' result rows, copied into the rows
                         // by the tile pass unless the solve is flagged (the
                         // rows keep their inputs for the exact sweeps)
    uint32_t gate;       // 0, or 1 + a result word: the solve runs only if that
                         // word is non-zero (a chained device elimination's
                         // outcome, GeDesc kGeChained: its rows and
                         // coefficients are what k_ge wrote)
    uint32_t pad;
};

/// Solves of up to this many rows may run as the product X = T R (their
/// inverse T = U^-1 L^-1 in scratch, rows of kTStride bytes), in split
/// launches (solve_split: the prefix pass is then its own launch).
constexpr unsigned kProductMaxRows = 120;
constexpr unsigned kSolvePrefixSplit = 16;
constexpr unsigned kSolveSplitMinRows = 16;
/// Whether a launch's solves take the split form (prefix pass and inverse,
/// product, copy-in: three launches) rather than k_solve_main's fused sweeps:
/// many solves, or any solve whose serial sweeps would outlast the three
/// launches (a lone 51-row solve: 209 us as sweeps, profiles/r6_kernel_stats).
constexpr bool solve_split(uint32_t solveCount, uint32_t maxRows)
{
    return solveCount >= kSolvePrefixSplit || maxRows >= kSolveSplitMinRows;
}
constexpr uint32_t kTStride = 128;
constexpr uint32_t solve_t_bytes(uint32_t m)
{
    return m <= kProductMaxRows ? ((m + 3u) & ~3u) * kTStride : 0u;
}
/// Row stride of the product solves' result scratch (64-byte chunks).
constexpr uint32_t solve_x_stride(uint32_t maxBytes) { return (maxBytes + 63u) & ~63u; }
constexpr uint64_t solve_x_bytes(uint32_t m, uint32_t maxBytes)
{
    return m <= kProductMaxRows ? (uint64_t)m * solve_x_stride(maxBytes) : 0u;
}

struct SolveRow
{
    uint64_t buf;        // recovery buffer (becomes the recovered original)
    uint32_t initBytes;  // Bytes before MultiplyLowerTriangle
    uint32_t lowerLen;   // Bytes when this row is the source of the lower step
    uint32_t finalBytes; // Bytes after MultiplyLowerTriangle
    uint32_t headIndex;  // 1 + the row's slot in SolveDesc.head (0: its own
                         // index; a chained elimination permutes the rows into
                         // pivot order after their heads were laid out)
};
constexpr uint32_t solve_head_slot(uint32_t headIndex, uint32_t j) { return headIndex ? headIndex - 1u : j; }

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

/// Ingest of a run of `count` symbols into FRESH device buffers (never
/// referenced by any op of the same flush before this point), so ingest can
/// run as the first launch of a flush.  Symbol k of the run (k < count; a
/// count of 0 reads as 1) has its source at src + k * srcStride and its
/// destination at dst + k * dstStride:  dst[0,hdrLen) = hdr,
/// dst[hdrLen, hdrLen+bytes) = src, and dst[total, align16(total)) = 0 (whole
/// 16-byte lanes are stored; dst is 16-byte aligned with capacity >=
/// align16(total)).  Bit k of dst2Mask set: symbol k is also written to the
/// fresh buffer dst2 + k * dstStride (an encoder and a decoder ingesting the
/// same originals: the source is read once; the decoder's lost originals
/// are the clear bits).  A run is a slab's consecutive slots filled from
/// consecutive device originals: one descriptor instead of one per symbol.
struct IngestDesc
{
    uint64_t dst;
    uint64_t src;
    uint64_t dst2;
    uint64_t dst2Mask;
    uint32_t bytes;
    uint32_t hdrLen;
    uint8_t hdr[8];
    uint32_t count;
    uint32_t srcStride;
    uint32_t dstStride;
    uint32_t pad;
};

/// Symbols of one ingest run at most (k_ingest block table: 4 bits of
/// 4-symbol groups per entry).
constexpr uint32_t kIngestRunMax = 64;
/// k_ingest work per workgroup: one symbol per wave.
constexpr uint32_t kIngestWaves = 4;

constexpr unsigned kTileBytes = 1024;       // solve tiles: 64 lanes x 16 bytes
constexpr unsigned kIngestChunkBytes = 8192;   // k_ingest: bytes per wave (8 x 1 KiB tiles)
/// Solves with more rows than this stage 256-byte tiles (16 lanes x 16 bytes
/// per row, four rows per wave) so all m <= 255 rows and the m x m
/// coefficients still fit one workgroup's LDS.
constexpr unsigned kSolveWideMaxRows = 120;
constexpr unsigned kSolveNarrowTileBytes = 256;
inline unsigned solve_tile_bytes(uint32_t m)
{
    return m > kSolveWideMaxRows ? kSolveNarrowTileBytes : kTileBytes;
}
/// Recovery-matrix generation + Gaussian elimination of one decode on the
/// device (k_ge; reference SiameseDecoder.cpp:2157-2531, the host's
/// generate_matrix + gaussian_elimination).  A job is a FRESH matrix of
/// `rows` recovery rows x `cols` lost columns (rows >= cols):
///   input (16-byte aligned, at GeDesc.in in the upload):
///     GeRow[rows], GeCol[cols], then pickLen bytes of pick columns: the
///     matrix column of window element pickLo + x (0xff: received);
///   output (GeDesc.result words of the result array, ge_result_words):
///     [0] the first pivot whose column has no non-zero left (== cols: the
///         matrix was eliminated), [1..2] the elimination's multiplied bytes
///         (the reference's muladds, u64), [3] 1 when [0] == cols, else 0,
///     [4] the non-zero coefficients below the diagonal of the eliminated
///         matrix in pivot order (MultiplyLowerTriangle's muladds per row
///         byte), [5..7] 0;
///     then the pivots (u8 row index per pivot position, padded to words);
///     without kGeChained also the used rows (u8 0/1), the column counts
///     (u16) and the matrix, rows x cols bytes in row order.
/// kGeChained (rows == cols): the decode's elimination of received data and
/// its solve were queued in the same submission, gated on word [3] (OP_ROWS
/// GfOp.termBegin, SolveDesc.gate).  On success the job writes the solve's
/// coefficients in pivot order (coef + solveCoef, cols x cols) and permutes
/// the solve's rows (rows + solveRow) into pivot order, each keeping its head
/// slot (SolveRow.headIndex).
/// Row kinds: Siamese (dense over [0, jEnd) from the row's opcodes, then
/// 2*ceil(ldpcN/16) PCG picks over [pickOff, pickOff + ldpcN)), Cauchy
/// (1/((rbase) ^ ccol) over [0, jEnd)) and parity (1 over [0, jEnd)).
struct GeDesc
{
    uint32_t in;        // byte offset of the job's input in the upload
    uint32_t result;    // first result word
    uint16_t rows, cols;
    uint32_t pickLen;
    uint32_t flags;     // kGeChained
    uint32_t solveRow;  // kGeChained: the solve's first SolveRow
    uint32_t solveCoef; // kGeChained: its coefficients' byte offset
    uint32_t pad;
};
static_assert(sizeof(GeDesc) == 32, "GeDesc layout");
constexpr uint32_t kGeChained = 1;

enum : uint8_t
{
    GE_SIAMESE = 0,
    GE_CAUCHY = 1,
    GE_PARITY = 2
};

struct GeRow
{
    uint16_t row;        // Siamese row number (opcodes, RX) / unused
    uint8_t kind;        // GE_*
    uint8_t rbase;       // Cauchy: (uint8)(row - 1 + kCauchyMaxColumns)
    uint16_t jEnd;       // dense columns [0, jEnd)
    uint16_t colCount;   // the row's column count (RecoveryPacket lost count)
    uint32_t ldpcN;      // Siamese: picks draw over ldpcN window elements
    uint32_t pickOff;    // ... starting at this index of the pick table
};

struct GeCol
{
    uint8_t lane;        // column % kLanes
    uint8_t cx, cx2;     // CX(column), CX(column)^2
    uint8_t ccol;        // column % kCauchyMaxColumns
};

/// Device elimination limits (LDS-resident matrix of one wave): the
/// reference's 255 lost columns (SiameseCommon.h:80, kMaximumLossRecoveryCount)
/// and up to 256 recovery rows.
constexpr unsigned kGeMaxCols = 255;
constexpr unsigned kGeMaxRows = 256;
constexpr unsigned kGeMaxPick = 65535;
constexpr uint8_t kGeNoColumn = 0xff;
/// k_ge's LDS row stride in dwords: odd, so the rows a wave's lanes own
/// start in different banks.
constexpr uint32_t ge_stride_words(uint32_t cols) { return ((cols + 3u) / 4u) | 1u; }

constexpr uint32_t ge_input_bytes(uint32_t rows, uint32_t cols, uint32_t pickLen)
{
    return (rows * 16u + cols * 4u + pickLen + 15u) & ~15u;
}
/// Word offsets of the output parts (ge_result_words: the total).
constexpr uint32_t kGeOutHeader = 8;
constexpr uint32_t ge_out_pivots(uint32_t) { return kGeOutHeader; }
constexpr uint32_t ge_out_used(uint32_t rows) { return kGeOutHeader + (rows + 3) / 4; }
constexpr uint32_t ge_out_counts(uint32_t rows) { return kGeOutHeader + 2 * ((rows + 3) / 4); }
constexpr uint32_t ge_out_matrix(uint32_t rows) { return ge_out_counts(rows) + (rows + 1) / 2; }
constexpr uint32_t ge_result_words(uint32_t rows, uint32_t cols, bool chained = false)
{
    return chained ? ge_out_used(rows) : ge_out_matrix(rows) + (rows * cols + 3) / 4;
}

constexpr uint32_t kNoRows = 0xffffffffu;   // be_launch_exec: no OP_ROWS in the launch
constexpr unsigned kExecTileBytes = 256;    // executor tiles: 64 lanes x 4 bytes

} // namespace sgpu
