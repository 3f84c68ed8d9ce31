/*
 * gqingest.h — host-side read ingest: BAM (BGZF) -> the SoA of gqpileup.h, and MD tag ->
 * MD events.  Plain C ABI over caller-owned output buffers (two phases: the library
 * reports sizes, the caller allocates, the library fills).
 *
 * Replaces (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):
 *   Read.loadReadRDDAndSequenceDictionaryFromBAM, samtools path + per-record filters
 *       reads/Read.scala:368-451 (filters :411-428)
 *   Read.fromSAMRecord (isMapped, sample name from the read group, 0-based start)
 *       reads/Read.scala:217-291
 *   ReadSet.mappedReads                                   ReadSet.scala:47-53
 *   MappedRead.end = start + cigar.getPaddedReferenceLength   reads/MappedRead.scala:87
 *   MappedRead.apply -> ADAM MdTag(md, start, cigar)       reads/MappedRead.scala:114-131
 * The BAM/BGZF decoding itself is htsjdk 1.118's SAMFileReader (pom.xml:317-321), written
 * here from the SAM/BAM format specification.
 *
 * Threading: every call takes n_threads (<= 0: the machine's hardware threads, at most 16).
 * Errors: a non-zero status and a thread-local message (gq_ingest_last_error).
 */
#ifndef GQINGEST_H
#define GQINGEST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  GQI_OK = 0,
  GQI_E_IO = 1,      /* open / read / mmap failed                                     */
  GQI_E_FORMAT = 2,  /* not BGZF / BAM, corrupt block (CRC / ISIZE), truncated record   */
  GQI_E_RECORD = 3,  /* ReadLoadError: bad aux type, base quality length != sequence   */
  GQI_E_MD = 4,      /* MdTag parse error (ADAM MdTag.apply)                            */
  GQI_E_ARG = 5,
  GQI_E_NOMEM = 6
} gqi_status;

const char *gq_ingest_last_error(void);

/* ---- BAM ------------------------------------------------------------------------------ */
typedef struct gq_bam gq_bam;

/* Maps the file and inflates every BGZF block (blocks in parallel; CRC32 and ISIZE checked).
 * A gzip stream without BGZF block sizes is inflated sequentially.                       */
gqi_status gq_bam_open(const char *path, int32_t n_threads, gq_bam **out);
void gq_bam_close(gq_bam *b);

/* Header: SAM text (NUL-terminated, trailing NULs stripped) and the reference dictionary. */
const char *gq_bam_header_text(const gq_bam *b);
int32_t gq_bam_n_contigs(const gq_bam *b);
const char *gq_bam_contig_name(const gq_bam *b, int32_t i);
int64_t gq_bam_contig_length(const gq_bam *b, int32_t i);

/* Read.InputFilters (reads/Read.scala:95-122).  Only mapped reads are returned
 * (ReadSet.mappedReads).  use_loci: the overlapsLoci filter; the loci of header contig c
 * are the sorted, disjoint half-open ranges [loci_begin[c], loci_begin[c+1]) of
 * loci_start / loci_end (a read is kept iff [pos, pos + reference length) intersects one). */
typedef struct {
  int32_t non_duplicate;
  int32_t passed_vendor_quality_checks;
  int32_t is_paired;
  int32_t has_md_tag;
  int32_t use_loci;
  const int64_t *loci_begin; /* [n_contigs + 1] */
  const int64_t *loci_start;
  const int64_t *loci_end;
} gq_bam_filters;

/* Sizes of the decoded, filtered read set (phase 1). */
typedef struct {
  int64_t n_reads;
  int64_t seq_bytes;  /* = qual bytes */
  int64_t cigar_len;  /* uint32 ops   */
  int64_t md_bytes;   /* MD strings   */
  int64_t name_bytes; /* read names   */
  int32_t n_rg;       /* distinct RG tag values among the kept reads, in order of first appearance */
  int32_t sorted;     /* the kept reads were already in (contig, start) order in the file        */
} gq_bam_sizes;

/* Decode every record (in parallel), apply the filters, and keep the result inside b.  */
gqi_status gq_bam_scan(gq_bam *b, const gq_bam_filters *f, int32_t n_threads, gq_bam_sizes *sizes);

/* RG value k (0 <= k < n_rg) of the last scan, and the file-order index (among the kept
 * reads) of its first read; k = -1: the first kept read without an RG tag (-1 if none).
 * Read.fromSAMRecord takes the sample name from the read group (reads/Read.scala:233-237);
 * the caller maps RG values to samples and numbers samples by first appearance.        */
const char *gq_bam_rg(const gq_bam *b, int32_t k);
int64_t gq_bam_rg_first(const gq_bam *b, int32_t k);

/* Output arrays (caller-owned, sized from gq_bam_sizes).  Reads are sorted by
 * (contig, start), ties in file order.  rg = index into gq_bam_rg, -1 = no RG tag.
 * md_len = -1 for a read without an MD tag.  flags bit0 = reverse strand.          */
typedef struct {
  int32_t *contig;
  int64_t *start, *end;
  uint8_t *mapq, *flags;
  int32_t *rg;
  int64_t *seq_off;
  int32_t *seq_len;
  uint8_t *seq, *qual;
  int64_t *cigar_off;
  int32_t *n_cigar;
  uint32_t *cigar;
  int64_t *md_off;
  int32_t *md_len;
  uint8_t *md;
  int64_t *name_off;
  int32_t *name_len;
  uint8_t *names;
} gq_bam_reads;

gqi_status gq_bam_fill(gq_bam *b, int32_t n_threads, const gq_bam_reads *out);

/* ---- MD tags -> MD events ---------------------------------------------------------------
 * ADAM MdTag(md, start, cigar) as MappedRead.apply builds it (reads/MappedRead.scala:130,
 * MDTagUtils.scala:23-78): digits = matching bases, letters = mismatches on M/=/X
 * positions, '^' + letters = deleted bases on D positions, N gaps skipped.
 * Event = (reference offset from the read start) << 8 | upper-case base, sorted by offset.
 * Phase 1 gives n_md (-1 for md_len < 0) and n_mismatch (saturated at 65535); the caller
 * sets md_ev_off = exclusive scan of max(n_md, 0); phase 2 writes the events.            */
gqi_status gq_md_count(int64_t n, const int64_t *cigar_off, const int32_t *n_cigar, const uint32_t *cigar,
                       const int64_t *md_off, const int32_t *md_len, const uint8_t *md, int32_t n_threads,
                       int32_t *n_md, uint16_t *n_mismatch);
gqi_status gq_md_fill(int64_t n, const int64_t *cigar_off, const int32_t *n_cigar, const uint32_t *cigar,
                      const int64_t *md_off, const int32_t *md_len, const uint8_t *md, const int64_t *md_ev_off,
                      int32_t n_threads, uint32_t *md_ev);

#ifdef __cplusplus
}
#endif
#endif
