/*
 * jwave_oracle_par.c — multi-core restatements of the reference's ForkJoin CPU
 * paths, for bench.py's cpu_baseline leg.
 *
 * TEST INFRASTRUCTURE ONLY (see jwave_oracle.c).  The per-line math is the
 * oracle's single-thread restatement; only the work split differs, the way
 * the reference's ForkJoinPool splits it:
 *  - ParallelTransform 2-D (ParallelTransform.java:70-126, tasks :222-330):
 *    forward = every row (lvlN), join, every column (lvlM); reverse = columns,
 *    join, rows.  Rows / columns are split into contiguous chunks, one per
 *    thread (the ForkJoin split bottoms out at 16 lines, :28, :243, :294; with
 *    8192 lines per pass a chunk per worker is the same work per core).
 *  - signal-level parallel batch (ParallelizationOpportunityTest.java:80-98):
 *    independent signals split over threads, each a sequential 1-D call.
 * Outputs are bit-identical to the sequential oracle (same per-line code).
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_taps orc_taps;
int orc_fwt_forward(const orc_taps* t, const double* x, double* y, int n, int level);
int orc_fwt_reverse(const orc_taps* t, const double* y, double* x, int n, int level);
int orc_wpt_forward(const orc_taps* t, const double* x, double* y, int n, int level);
int orc_wpt_reverse(const orc_taps* t, const double* y, double* x, int n, int level);

typedef int (*line_fn)(const orc_taps*, const double*, double*, int, int);

static line_fn pick_fn(int kind, int forward) {
  if (kind == 0) return forward ? orc_fwt_forward : orc_fwt_reverse;
  return forward ? orc_wpt_forward : orc_wpt_reverse;
}

typedef struct {
  line_fn fn;
  const orc_taps* t;
  const double* src;
  double* dst;
  int rows, cols, lvl_m, lvl_n, forward;
  int id, nth;
  pthread_barrier_t* bar;
  int rc;
} job2d;

static int rows_pass(job2d* j, const double* src, double* dst) {
  const int r0 = (int)((int64_t)j->rows * j->id / j->nth);
  const int r1 = (int)((int64_t)j->rows * (j->id + 1) / j->nth);
  double* b = (double*)malloc(sizeof(double) * (size_t)j->cols);
  int rc = 0;
  for (int i = r0; i < r1 && !rc; i++) {
    rc = j->fn(j->t, src + (size_t)i * j->cols, b, j->cols, j->lvl_n);
    memcpy(dst + (size_t)i * j->cols, b, sizeof(double) * (size_t)j->cols);
  }
  free(b);
  return rc;
}

/* column gather -> transform -> scatter (ParallelTransform's column tasks
 * copy matrix[j][col] into a fresh array the same way) */
static int cols_pass(job2d* j, const double* src, double* dst) {
  const int c0 = (int)((int64_t)j->cols * j->id / j->nth);
  const int c1 = (int)((int64_t)j->cols * (j->id + 1) / j->nth);
  double* a = (double*)malloc(sizeof(double) * (size_t)j->rows);
  double* b = (double*)malloc(sizeof(double) * (size_t)j->rows);
  int rc = 0;
  for (int c = c0; c < c1 && !rc; c++) {
    for (int i = 0; i < j->rows; i++) a[i] = src[(size_t)i * j->cols + c];
    rc = j->fn(j->t, a, b, j->rows, j->lvl_m);
    for (int i = 0; i < j->rows; i++) dst[(size_t)i * j->cols + c] = b[i];
  }
  free(a);
  free(b);
  return rc;
}

static void* work2d(void* p) {
  job2d* j = (job2d*)p;
  if (j->forward) {
    j->rc = rows_pass(j, j->src, j->dst);
    pthread_barrier_wait(j->bar);
    if (!j->rc) j->rc = cols_pass(j, j->dst, j->dst);
  } else {
    j->rc = cols_pass(j, j->src, j->dst);
    pthread_barrier_wait(j->bar);
    if (!j->rc) j->rc = rows_pass(j, j->dst, j->dst);
  }
  return NULL;
}

int orc_2d_par(int kind, int forward, const orc_taps* t, const double* x, double* y, int rows,
               int cols, int lvl_m, int lvl_n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  job2d* jobs = (job2d*)calloc((size_t)nthreads, sizeof(job2d));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
  for (int i = 0; i < nthreads; i++) {
    job2d j = {pick_fn(kind, forward), t, x, y, rows, cols, lvl_m, lvl_n, forward, i, nthreads,
               &bar, 0};
    jobs[i] = j;
    pthread_create(&th[i], NULL, work2d, &jobs[i]);
  }
  int rc = 0;
  for (int i = 0; i < nthreads; i++) {
    pthread_join(th[i], NULL);
    if (jobs[i].rc) rc = jobs[i].rc;
  }
  pthread_barrier_destroy(&bar);
  free(th);
  free(jobs);
  return rc;
}

typedef struct {
  line_fn fn;
  const orc_taps* t;
  const double* x;
  double* y;
  int batch, n, level, id, nth;
  int64_t ld;
  int rc;
} jobb;

static void* workb(void* p) {
  jobb* j = (jobb*)p;
  const int b0 = (int)((int64_t)j->batch * j->id / j->nth);
  const int b1 = (int)((int64_t)j->batch * (j->id + 1) / j->nth);
  for (int b = b0; b < b1 && !j->rc; b++)
    j->rc = j->fn(j->t, j->x + (size_t)b * j->ld, j->y + (size_t)b * j->ld, j->n, j->level);
  return NULL;
}

int orc_batch_par(int kind, int forward, const orc_taps* t, const double* x, double* y, int batch,
                  int n, int64_t ld, int level, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  jobb* jobs = (jobb*)calloc((size_t)nthreads, sizeof(jobb));
  for (int i = 0; i < nthreads; i++) {
    jobb j = {pick_fn(kind, forward), t, x, y, batch, n, level, i, nthreads, ld, 0};
    jobs[i] = j;
    pthread_create(&th[i], NULL, workb, &jobs[i]);
  }
  int rc = 0;
  for (int i = 0; i < nthreads; i++) {
    pthread_join(th[i], NULL);
    if (jobs[i].rc) rc = jobs[i].rc;
  }
  free(th);
  free(jobs);
  return rc;
}
