/*
 * gqpileup.h — C-ABI drop-in boundary of the MI355X pileup engine.
 *
 * Replaces, for the two callers named by BASELINE.json's north_star, the Spark
 * operator + per-locus callback pair of the reference (paths relative to
 * /root/reference/src/main/scala/org/hammerlab/guacamole/):
 *
 *   DistributedUtil.pileupFlatMap[T](reads, lociPartitions, skipEmpty, function, reference)
 *       DistributedUtil.scala:288-306
 *   DistributedUtil.pileupFlatMapTwoRDDs[T](reads1, reads2, lociPartitions, skipEmpty, function, ref)
 *       DistributedUtil.scala:316-335
 *   GermlineThreshold.Caller.callVariantsAtLocus(pileup, thresholdPercent, emitRef, emitNoCall)
 *       commands/GermlineThresholdCaller.scala:90-179
 *   SomaticStandard.Caller.findPotentialVariantAtLocus(tumor, normal, odds, minMapq, multiAllelic, maxDepth)
 *       commands/SomaticStandardCaller.scala:162-245  (+ driver filters :124-151)
 *
 * A JVM closure cannot cross a C ABI, so operator + callback are fused into
 * fixed-function entry points (gq_germline_threshold, gq_somatic_standard) and
 * a raw per-locus histogram (gq_pileup_counts).  skipEmpty = true is the only
 * mode (both callers pass true: GermlineThresholdCaller.scala:76,
 * SomaticStandardCaller.scala:108).
 *
 * Conventions: plain pointers + sizes, no exceptions across the ABI.  Every
 * function returns a gq_status; gq_last_error() gives the thread-local message.
 * Read sets are uploaded once to HBM (gq_reads_upload) and stay resident; the
 * caller owns host buffers, the library owns device memory and result buffers
 * (released with gq_free_calls / gq_free_somatic / gq_free_counts).
 * One gq_ctx per device; calls on a context are serialized (not re-entrant);
 * contexts on different devices may run concurrently from different threads.
 */
#ifndef GQPILEUP_H
#define GQPILEUP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes mirror the reference's exception classes. */
typedef enum {
  GQ_OK = 0,
  GQ_E_ASSERT = 1,          /* assume/assert failures (AssertionError)                    */
  GQ_E_INVALID_CIGAR = 2,   /* InvalidCigarElementException  PileupElement.scala:277-285   */
  GQ_E_MD = 3,              /* CigarMDTagMismatchException   MappedRead.scala:138-139     */
  GQ_E_NO_MD = 4,           /* ReferenceWithoutMDTagException MappedRead.scala:141        */
  GQ_E_MULTI_REF = 5,       /* "Multiple reference bases found" GermlineThresholdCaller:171 */
  GQ_E_UNSORTED = 6,        /* "Regions must be sorted"       SlidingWindow.scala:55-56   */
  GQ_E_ARG = 7,             /* IllegalArgumentException (bad arguments / loci)             */
  GQ_E_HIP = 8,             /* device runtime error                                       */
  GQ_E_NOMEM = 9,
  GQ_E_CAPACITY = 10,       /* a per-locus table overflowed (distinct alleles > capacity)  */
  /* gq_bam_dev_* (BAM decoded on the device), the host loader's gqi_status classes:          */
  GQ_E_BAM_IO = 11,         /* open / stat / map failed                        (GQI_E_IO)     */
  GQ_E_BAM_FORMAT = 12,     /* not BAM, corrupt BGZF block, truncated record   (GQI_E_FORMAT) */
  GQ_E_BAM_RECORD = 13,     /* ReadLoadError: bad aux type, missing qualities  (GQI_E_RECORD) */
  GQ_E_MD_PARSE = 14,       /* MdTag parse error (ADAM MdTag.apply)            (GQI_E_MD)     */
  GQ_E_NOT_BGZF = 15,       /* a gzip stream without BGZF block sizes: use the host loader    */
  GQ_E_PLAN = 16            /* a region plan (gq_bam_dev_plan) does not hold for this file:   */
                            /* not coordinate-sorted, or a record runs past a planned segment */
                            /* (load the whole file instead)                                  */
} gq_status;

/* CIGAR ops use BAM packing: len << 4 | op, op in M I D N S H P = X -> 0..8. */

/* Read set, structure-of-arrays.  Reads are sorted by (contig, start), ties in
 * input (file) order; contig c owns reads [contig_read_begin[c], contig_read_begin[c+1]).
 * Coordinates are 0-based, contig-relative.  MD tags are pre-parsed into events:
 * md_ev[i] = (offset from read start) << 8 | base, sorted by offset, covering both
 * mismatches (on M/=/X positions) and deleted bases (on D positions).         */
typedef struct {
  int64_t n_reads;
  int32_t n_contigs;
  int32_t n_samples;
  const int64_t *contig_read_begin; /* [n_contigs + 1]                                */
  const int32_t *start;             /* [n_reads] alignment start                       */
  const int32_t *end;               /* [n_reads] start + padded reference length       */
  const int32_t *pmax_end;          /* [n_reads] prefix max of end within the contig   */
  const uint8_t *mapq;              /* [n_reads]                                       */
  const uint8_t *flags;             /* [n_reads] bit0 = reverse strand                 */
  const uint8_t *sample;            /* [n_reads] sample slot                           */
  const int64_t *seq_off;           /* [n_reads] offset into seq / qual pools          */
  const int32_t *seq_len;           /* [n_reads]                                       */
  const int64_t *cigar_off;         /* [n_reads]                                       */
  const int32_t *n_cigar;           /* [n_reads]                                       */
  const int64_t *md_off;            /* [n_reads]                                       */
  const int32_t *n_md;              /* [n_reads] MD events; -1 => read has no MD tag   */
  const uint16_t *n_mismatch;       /* [n_reads] MdTag.countOfMismatches               */
  int64_t seq_bytes;                /* pool sizes                                      */
  int64_t cigar_len;
  int64_t md_len;
  const uint8_t *seq;               /* ASCII bases                                     */
  const uint8_t *qual;              /* phred, same offsets as seq                      */
  const uint32_t *cigar;
  const uint32_t *md_ev;
  /* [n_samples] java.lang.String.hashCode of each slot's sample name (the JVM host passes
   * name.hashCode(); a read without a read group is sample "default", Pileup.scala:58), or
   * NULL.  It orders the per-sample records of a locus as Pileup.bySample's Scala Map iterates
   * (GermlineThresholdCaller.scala:100); NULL keeps slot order.                            */
  const uint32_t *sample_hash;
} gq_reads;

/* LociMap[Long] as flat ranges in partition order (task ascending, contigs
 * lexicographic, start ascending); half-open [start, end).                    */
typedef struct {
  int64_t n_ranges;
  const int32_t *contig;
  const int64_t *start;
  const int64_t *end;
  const int64_t *task;
} gq_loci;

typedef struct {
  int32_t threshold;    /* --threshold (default 8)   */
  int32_t emit_ref;     /* --emit-ref                */
  int32_t emit_no_call; /* --emit-no-call            */
} gq_germline_params;

/* GenotypeAllele codes (bdg-formats): */
enum { GQ_GT_REF = 0, GQ_GT_ALT = 1, GQ_GT_OTHERALT = 2, GQ_GT_NOCALL = 3 };
/* per-call flags (somatic calls: bit0 / bit1 = tumor / normal reference base
 * ambiguous, plus GQ_FLAG_KNIFE_EDGE) */
enum {
  GQ_FLAG_AMBIGUOUS_REF = 1, /* pileup ref base decided by JVM heap order (MD tags disagree) */
  GQ_FLAG_TIE = 2,           /* count tie among passing alleles, ordered as the reference's
                                Scala 2.10 groupBy map iterates (restated, parity unpinned) */
  GQ_FLAG_KNIFE_EDGE = 4     /* somatic: a test or filter decided within FP rounding of its
                                threshold (outcome depends on summation order)              */
};

/* Germline genotype records (Genotype.newBuilder, GermlineThresholdCaller.scala:106-117),
 * in output order (partition order, then sample, then allele rank).          */
typedef struct {
  int64_t n;
  int32_t *contig;
  int64_t *pos;
  uint8_t *sample;
  uint8_t *gt0, *gt1;
  uint8_t *flags;
  int64_t *ref_off;  int32_t *ref_len;   /* into allele_pool */
  int64_t *alt_off;  int32_t *alt_len;
  uint8_t *allele_pool;
  int64_t pool_len;
  /* run counters */
  int64_t visited_loci;   /* loci with depth > 0 (skipEmpty semantics)         */
  int64_t complex_loci;   /* loci routed through the general-allele kernel     */
  int64_t ambiguous_loci; /* loci whose ref base depends on heap order         */
  int64_t tie_loci;
  void *block_;           /* owner of the arrays above (freed by gq_free_calls) */
} gq_calls;

/* The same records left in HBM (gq_germline_threshold_device): `calls` holds DEVICE pointers
 * into one contiguous image owned by the context and valid until its next call (do not pass
 * it to gq_free_calls).  Image layout: int64 pool_len at byte 0, then the arrays of `calls`
 * in the order contig, pos, ref_off, alt_off, ref_len, alt_len, sample, gt0, gt1, flags, pool,
 * each starting on a 64-byte boundary (the first at byte 64); image_bytes covers the pool's
 * used bytes.  One buffer per rank is what the multi-GPU gather moves over xGMI.           */
typedef struct {
  gq_calls calls;
  const void *image;
  int64_t image_bytes;
} gq_calls_device;

typedef struct gq_ctx gq_ctx;
typedef struct gq_dev_reads gq_dev_reads;

/* Per-kernel device times of the last call on this context (HIP events on the
 * context's stream), in milliseconds. */
typedef struct {
  float plan_ms;
  float pileup_ms;   /* dominant kernel: per-tile LDS histogram + on-device decision */
  float complex_ms;
  float finalize_ms; /* sort / compaction of the call records                        */
  float total_ms;    /* first event to last event                                    */
  int64_t pileup_launches;
  int64_t tiles;
  float host_ms;     /* host wall time of the whole call (enqueue + waits + marshalling) */
  float marshal_ms;  /* host time spent building the output arrays                      */
  float walk_ms;     /* germline: the walker kernel over the tiles the column kernel     */
                     /* handed over (pileup_ms is then the column kernel alone)          */
  int64_t walk_tiles;
  int64_t order_loci;  /* germline: loci whose records depend on the restated Scala map order */
  int64_t deep_loci;   /* somatic: candidates the deep caller took (pileup past the fast path) */
  int64_t deep_max;    /* somatic: deepest per-sample pileup among them                     */
  float call_ms;       /* somatic: the fast exact-caller kernel alone (inside complex_ms)    */
  float deep_ms;       /* somatic: the deep caller launches (inside complex_ms)              */
  float front_ms;      /* somatic: the split caller's front kernel (covers + element records, */
                       /* inside call_ms)                                                     */
} gq_timings;

const char *gq_version(void);
const char *gq_last_error(void);

gq_status gq_open(int device, gq_ctx **out);
void gq_close(gq_ctx *ctx);
gq_status gq_get_timings(const gq_ctx *ctx, gq_timings *out);
/* Tile size (loci per workgroup) used by the pileup kernel; 0 => default. */
gq_status gq_set_tile(gq_ctx *ctx, int32_t loci_per_tile);

/* Copy a host read set into HBM (SoA kept resident until gq_reads_free).     */
gq_status gq_reads_upload(gq_ctx *ctx, const gq_reads *host, gq_dev_reads **out);
/* Wrap read arrays that are ALREADY in device memory (e.g. torch tensors);  */
/* the caller keeps them alive.                                              */
gq_status gq_reads_wrap_device(gq_ctx *ctx, const gq_reads *device_ptrs, gq_dev_reads **out);
void gq_reads_free(gq_dev_reads *r);
/* Drop every structure derived from a resident read set (the upload-time derivation, the     */
/* projection, the margin projection) and derive the upload-time part again; the projection  */
/* is derived again by the next call that reads it.  The SoA arrays stay resident and are not */
/* read from the host again; the derived buffers are reused.  A cold pass over reads already  */
/* in HBM: what one MappedRead RDD costs the reference per job, whose pileups are rebuilt by  */
/* every pileupFlatMap (DistributedUtil.scala:288-306; GermlineThresholdCaller.scala:58-88).  */
gq_status gq_reads_rederive(gq_ctx *ctx, gq_dev_reads *r);
/* Sizes of a resident read set and of what the upload derived from it (the germline         */
/* projection pool and its sparse entries): for measurement and capacity planning.             */
typedef struct gq_reads_info {
  int64_t n_reads, seq_bytes, proj_bytes, pev_count, proj_reads;  /* proj_reads: reads the projection takes */
  int64_t n_rows;    /* projection rows (64 bytes each: proj_bytes = 64 n_rows) */
  float h2d_ms;      /* gq_reads_upload: host wall time of the copies (pinned staging, PCIe) */
  float derive_ms;   /* gq_reads_upload / wrap: the upload-time derivation on the device    */
  int64_t cigar_len, md_len;  /* pool sizes (CIGAR ops, MD events) */
  int32_t n_contigs, n_samples;
  float proj_ms;     /* the projection, derived on the first call that reads it (0: not yet) */
  int32_t projected; /* 1 once it is: the proj_* / n_rows / pev_count sizes above are then set */
  float fill_ms;       /* its pool fill kernel(s) (HIP events on the context's stream) */
  float proj_dev_ms;   /* its device span, first kernel to last (HIP events) */
  float derive_dev_ms; /* the upload-time derivation's device span (HIP events) */
} gq_reads_info;
/* A re-derivation and a projection do not wait for their device spans: this call waits for   */
/* them (and reads the projection's taken-read count) the first time it is asked after them;  */
/* the next re-derivation drops figures nobody asked for.                                      */
gq_status gq_reads_get_info(const gq_dev_reads *r, gq_reads_info *out);

/* ---- BAM decoded on the device ----------------------------------------------------------
 * The host loader of gqingest.h (Read.loadReadRDDAndSequenceDictionaryFromBAM and its
 * filters, reads/Read.scala:368-451 / :411-428; Read.fromSAMRecord :217-291;
 * ReadSet.mappedReads ReadSet.scala:47-53; MappedRead.end :87; the MdTag of
 * MappedRead.apply :114-131) with every step after the file read in HBM: the BGZF blocks are
 * inflated on the device (CRC32 and ISIZE checked), record boundaries found there, each record
 * parsed and filtered, MD tags turned into events, and the kept reads laid out as a resident
 * gq_dev_reads.  The compressed file is the only host -> device copy.  Same rules, same
 * arrays as gq_bam_open / gq_bam_scan / gq_bam_fill + gq_md_count / gq_md_fill + upload.
 *   open  -> header (text, reference dictionary) on the host, inflated stream in HBM
 *   scan  -> filters, sizes, the read-group classes' first kept records (the caller maps
 *            read groups to samples, numbered by first appearance: Read.scala:233-237)
 *   reads -> the resident read set (GQ_E_UNSORTED if the kept reads are not in (contig,
 *            start) order: the host loader sorts such files)                               */
typedef struct gq_bam_dev gq_bam_dev;

gq_status gq_bam_dev_open(gq_ctx *ctx, const char *path, gq_bam_dev **out);
/* gq_bam_dev_open in two steps: map (host only: the file, its BGZF block table and the header,
 * inflated on the host; may run while the device context starts) and load (copy, inflate) on
 * a context.  gq_bam_dev_map_ex(populate = 0) maps without faulting the whole file in (for a
 * region-restricted load, which reads only its segments' pages).                            */
gq_status gq_bam_dev_map(const char *path, gq_bam_dev **out);
gq_status gq_bam_dev_map_ex(const char *path, int32_t populate, gq_bam_dev **out);
gq_status gq_bam_dev_load(gq_ctx *ctx, gq_bam_dev *mapped);

/* Region-restricted load (the multi-GPU ingest): one rank reads only the records that can
 * overlap its loci — the reads the reference ships to that rank's tasks
 * (DistributedUtil.scala:584-597; the whole-file read Read.scala:368-451 is what it replaces
 * at world size > 1).  Host only, before gq_bam_dev_load.  Loci: per contig of the BAM's
 * dictionary, sorted disjoint half-open ranges (loci_begin[n_contigs + 1] indexes
 * loci_start / loci_end, as gq_bam_dev_filters).  Each range's records are found
 *   * from the BAI linear index (`bai_path`; NULL or "" for none): the first record that can
 *     overlap the range's first locus (exact for any read length); or, without an index,
 *     by host probes of BGZF blocks (binary search over the blocks' last record keys), from
 *     `halo` loci before the range;
 *   * up to the first BGZF block whose records all start at or past the range's end (probes).
 * Ranges whose blocks meet are merged into one segment.  The next gq_bam_dev_load copies and
 * inflates only the segments' blocks; gq_bam_dev_scan walks each segment's records from its
 * first record.  GQ_E_PLAN: the header does not declare SO:coordinate, or the index does not
 * fit the file (then load the whole file).                                                  */
typedef struct {
  int64_t n_segments;
  int64_t n_blocks;        /* BGZF blocks the load will inflate                                  */
  int64_t comp_bytes;      /* their compressed bytes (the load's host -> device copy)          */
  int64_t bam_bytes;       /* their inflated bytes                                             */
  int64_t probes;          /* host probes (blocks inflated on the host to read record keys)    */
  int32_t used_index;      /* 1: range starts from the BAI linear index                        */
  int32_t pad;
} gq_bam_dev_plan_info;
gq_status gq_bam_dev_plan(gq_bam_dev *b, const int64_t *loci_begin, const int64_t *loci_start,
                          const int64_t *loci_end, int64_t halo, const char *bai_path,
                          gq_bam_dev_plan_info *info);
/* The planned segments (n_segments entries each): first BGZF block, offset of the first record
 * in that block's inflated bytes, end block (exclusive), and whether records run to the end of
 * the file (else block end - 1 is read only to complete the last record before it).         */
gq_status gq_bam_dev_plan_segments(const gq_bam_dev *b, int64_t *first_block, int64_t *first_offset,
                                   int64_t *end_block, int32_t *to_eof);
void gq_bam_dev_close(gq_bam_dev *b);
const char *gq_bam_dev_header_text(const gq_bam_dev *b); /* SAM text, trailing NULs stripped */
int32_t gq_bam_dev_n_contigs(const gq_bam_dev *b);
const char *gq_bam_dev_contig_name(const gq_bam_dev *b, int32_t i);
int64_t gq_bam_dev_contig_length(const gq_bam_dev *b, int32_t i);

typedef struct {
  int32_t non_duplicate;   /* Read.InputFilters, as gqingest.h gq_bam_filters                   */
  int32_t passed_vendor_quality_checks;
  int32_t is_paired;
  int32_t has_md_tag;
  int32_t use_loci;
  const int64_t *loci_begin; /* [n_contigs + 1] */
  const int64_t *loci_start;
  const int64_t *loci_end;
  int32_t n_rg;            /* the header's @RG IDs: n_rg NUL-terminated strings back to back */
  const char *rg_ids;
} gq_bam_dev_filters;

typedef struct {
  int64_t n_records;       /* alignment records in the file */
  int64_t n_reads;         /* kept                          */
  int64_t seq_bytes, cigar_len, md_events;
  int64_t comp_bytes, bam_bytes; /* compressed file / inflated stream */
  int64_t n_blocks;        /* BGZF blocks                   */
  float map_ms, h2d_ms, inflate_ms, records_ms, parse_ms;  /* open: map + block walk, copy, inflate; scan */
  int64_t max_span;        /* largest reference span (end - start) of a mapped record scanned  */
} gq_bam_dev_sizes;

/* rg_first[k] (k < n_rg): file-order index of the first kept record whose RG tag is header ID
 * k; rg_first[n_rg]: of the first kept record without an RG tag or with an ID the header
 * lacks (both are sample "default"); -1 where none.                                         */
gq_status gq_bam_dev_scan(gq_bam_dev *b, const gq_bam_dev_filters *f, int64_t *rg_first, gq_bam_dev_sizes *sizes);
/* class_sample[k] (k <= n_rg): the sample slot of read-group class k; sample_hash as in
 * gq_reads, may be NULL.  The handle is independent of b (b may be closed after).          */
gq_status gq_bam_dev_reads(gq_bam_dev *b, const uint8_t *class_sample, int32_t n_samples,
                           const uint32_t *sample_hash, gq_dev_reads **out, float *fill_ms);

/* Copies out of a resident read set (host buffers of n_reads / n_contigs + 1 entries).      */
gq_status gq_reads_positions(const gq_dev_reads *r, int32_t *start, int32_t *end);
gq_status gq_reads_contig_begin(const gq_dev_reads *r, int64_t *out);
/* The whole SoA of a resident read set copied into host buffers (dst's pointers, sized from
 * gq_reads_info; a NULL pointer is skipped): the parity tests compare it with the host loader. */
gq_status gq_reads_download(const gq_dev_reads *r, const gq_reads *dst);

/* germline-threshold over the given loci partitions.                         */
gq_status gq_germline_threshold(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci,
                                const gq_germline_params *params, gq_calls **out);
void gq_free_calls(gq_calls *c);
/* The body of the VCF a germline-threshold run writes (Common.scala:290-293 saveAsVcf of the
 * records' single sample: "CHROM POS . REF ALT . . . GT <gt>" per record, POS 1-based) after
 * `header` (the ## lines and the #CHROM line), to `path`; contig_names[k] names contig id k.
 * GQ_E_ARG on an unwritable path.  The CLI's writer for one-sample output (Python builds the
 * multi-sample layout).                                                                     */
gq_status gq_write_vcf_germline(const char *path, const char *header, int64_t n, const int32_t *contig,
                                const int64_t *pos, const uint8_t *gt0, const uint8_t *gt1, const int64_t *ref_off,
                                const int32_t *ref_len, const int64_t *alt_off, const int32_t *alt_len,
                                const uint8_t *pool, int32_t n_contigs, const char *const *contig_names);
/* gq_germline_threshold with the records left in HBM (no PCIe copy; the multi-GPU driver
 * gathers the images over xGMI).  Same decisions, same record order.                      */
gq_status gq_germline_threshold_device(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci,
                                       const gq_germline_params *p, gq_calls_device *out);

/* Raw per-locus pileup histogram for every locus of `loci` (dense, in range
 * order).  Categories: Match/Mismatch by sequenced base A,C,G,T,N,other; then
 * insertion, deletion, mid-deletion, clipped; positive-strand depth; the
 * MD-derived reference base (or 'N'); ambiguous-ref flag.                     */
typedef struct {
  int64_t n_loci;
  int32_t *depth;
  int32_t *pos_depth;
  int32_t *base_counts;   /* [n_loci * 6]  A C G T N other              */
  int32_t *indel_counts;  /* [n_loci * 4]  ins del middel clipped       */
  int32_t *ref_depth;     /* Match elements                             */
  uint8_t *ref_base;
  uint8_t *ambiguous;
} gq_counts;
gq_status gq_pileup_counts(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci, gq_counts **out);
void gq_free_counts(gq_counts *c);

/* somatic-standard.                                                          */
typedef struct {
  int32_t odds;                 /* --odds (20)                          */
  int32_t min_mapq;             /* --min-mapq (1)                       */
  int32_t filter_multi_allelic; /* --filter-multi-allelic               */
  int32_t max_read_depth;       /* caller's maxReadDepth (= --max-tumor-read-depth) */
  int32_t min_tumor_read_depth, max_tumor_read_depth, min_normal_read_depth;
  int32_t min_tumor_alternate_read_depth;
  int32_t min_lod, min_likelihood, min_vaf;
  int32_t min_average_mapping_quality, min_average_base_quality;
  int32_t max_median_mismatches;
  int32_t apply_filters;        /* 0 => raw findPotentialVariantAtLocus output */
} gq_somatic_params;

typedef struct {
  double likelihood;
  int32_t read_depth, allele_read_depth, forward_depth, allele_forward_depth;
  double mean_mq, median_mq, mean_bq, median_bq, median_mismatches;
} gq_evidence;

/* CalledSomaticAllele (variants/CalledSomaticAllele.scala:37-51)            */
typedef struct {
  int64_t n;
  int32_t *contig;
  int64_t *pos;
  uint8_t *sample;
  int64_t *ref_off;  int32_t *ref_len;
  int64_t *alt_off;  int32_t *alt_len;
  uint8_t *allele_pool;
  int64_t pool_len;
  double *log_odds;
  int32_t *gq;               /* phredScaledSomaticLikelihood                 */
  gq_evidence *tumor;        /* tumorVariantEvidence                         */
  gq_evidence *normal;       /* normalReferenceEvidence                      */
  uint8_t *flags;
  int64_t visited_loci;
  int64_t candidate_loci;    /* loci that reached the likelihood kernel      */
  void *block_;              /* owner of the arrays above when non-NULL (freed by gq_free_somatic) */
} gq_somatic_calls;

gq_status gq_somatic_standard(gq_ctx *ctx, const gq_dev_reads *tumor, const gq_dev_reads *normal,
                              const gq_loci *loci, const gq_somatic_params *params, gq_somatic_calls **out);
void gq_free_somatic(gq_somatic_calls *c);

/* variant-support: VariantSupport.pileupToAlleleCounts (commands/VariantSupport.scala:110-118)
 * over pileupFlatMap(reads, partitions, skipEmpty = true, ...) (:93-100).  One row per
 * (visited locus, distinct allele of its pileup): every element counts (no filter).  Rows in
 * call order of the loci, a locus's alleles by (ref, alt) bytes (the reference iterates a Scala
 * HashMap there: order unpinned).  sample = the pileup's head-element read sample
 * (Pileup.scala:51); flags bit0 = reference base from heap order (MD tags disagree), bit1 =
 * the pileup mixes samples (the head element, hence `sample`, is then heap-order dependent). */
typedef struct {
  int64_t n;
  int32_t *contig;
  int64_t *pos;
  int32_t *sample;
  int32_t *count;
  int64_t *ref_off;  int32_t *ref_len;
  int64_t *alt_off;  int32_t *alt_len;
  uint8_t *allele_pool;
  int64_t pool_len;
  uint8_t *flags;
} gq_allele_counts;
gq_status gq_variant_support(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci, gq_allele_counts **out);
void gq_free_allele_counts(gq_allele_counts *c);

/* germline-standard: GermlineStandard.Caller.callVariantsAtLocus (commands/GermlineStandardCaller
 * .scala:90-124) over pileupFlatMap(reads, partitions, skipEmpty = true) (:63-68), then
 * GenotypeFilter (filters/GenotypeFilter.scala:140-154) when apply_filters.  Results in a
 * gq_somatic_calls: one row per CalledAllele, `sample` its sample slot, `tumor` its
 * AlleleEvidence, `gq` its phredScaledLikelihood, `normal` and `log_odds` zero; flags bit0 =
 * the pileup reference base came from heap order.  A sample's rows follow sample order (the
 * reference iterates a Scala Map there: unpinned for > 1 sample).                          */
typedef struct {
  int32_t min_mapq;                 /* --min-mapq (1): QualityAlignedReadsFilter        */
  int32_t min_read_depth;           /* --min-read-depth (0)                             */
  int32_t max_read_depth;           /* --max-read-depth (Int.MaxValue)                  */
  int32_t min_alternate_read_depth; /* --min-alternate-read-depth (0)                   */
  int32_t min_likelihood;           /* --min-likelihood (0)                             */
  int32_t apply_filters;            /* 0 => raw callVariantsAtLocus output              */
} gq_germline_std_params;
gq_status gq_germline_standard(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci,
                               const gq_germline_std_params *params, gq_somatic_calls **out);

/* vaf-histogram: VAFHistogram.variantLociFromReads + generateVAFHistogram
 * (commands/VAFHistogram.scala:208-229, 188-196): at every visited locus whose pileup holds a
 * non-Match element (VariantLocus.apply, :31-37), VAF = (depth - referenceDepth).toFloat /
 * depth; kept when depth >= min_read_depth and VAF >= min_vaf / 100.0; binned as
 * pct - pct % (100 / bins) with pct = (int)(VAF * 100).  counts[b] = loci in the bin starting
 * at b.  GQ_E_ASSERT unless 1 <= bins <= 100 (the reference's assume).                      */
typedef struct {
  int32_t bins;            /* --bins (20)          */
  int32_t min_read_depth;  /* --min-read-depth (0) */
  int32_t min_vaf;         /* --min-vaf (0)        */
} gq_vaf_params;
typedef struct {
  int64_t counts[101];
  int64_t variant_loci;  /* loci binned          */
  int64_t visited_loci;  /* non-empty pileups    */
} gq_vaf_hist;
gq_status gq_vaf_histogram(gq_ctx *ctx, const gq_dev_reads *reads, const gq_loci *loci, const gq_vaf_params *params,
                           gq_vaf_hist *out);

/* --reference-fasta (SomaticStandardCaller.scala:57, :75).  A reference genome resident in HBM
 * (replaces ReferenceBroadcast.apply, reference/ReferenceBroadcast.scala:39-55): bases[k] /
 * lengths[k] are the unmasked bases of contig k of the read sets' contig list (bases[k] == NULL
 * for a contig the FASTA lacks).  Bytes are copied; the caller's buffers may be freed after. */
typedef struct gq_reference gq_reference;
gq_status gq_reference_upload(gq_ctx *ctx, int32_t n_contigs, const uint8_t *const *bases, const int64_t *lengths,
                              gq_reference **out);
void gq_reference_free(gq_reference *ref);
/* gq_somatic_standard with pileupFlatMapTwoRDDs' referenceGenome argument
 * (DistributedUtil.scala:316-335): every pileup's reference base is the reference's
 * (DistributedUtil.scala:266-268) instead of the reads' MD-derived one.  ref == NULL is
 * gq_somatic_standard.  GQ_E_ARG when a loci range lies on a contig the reference lacks
 * (ContigNotFound, ReferenceBroadcast.scala:26-30) or runs past its end.               */
gq_status gq_somatic_standard_ref(gq_ctx *ctx, const gq_dev_reads *tumor, const gq_dev_reads *normal,
                                  const gq_loci *loci, const gq_reference *ref, const gq_somatic_params *params,
                                  gq_somatic_calls **out);

#ifdef __cplusplus
}
#endif
#endif
