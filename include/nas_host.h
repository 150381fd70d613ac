/* nas_host.h -- C ABI of the C++ host mirror (libnas_host.so), the layer
 * above include/nas.h that restates the reference's Go host
 * (scheduler/scheduler.go): metric ingest with Go's parsing semantics, the
 * iperf3 report decode, the pairwise latency matrix, and the CustomScheduler
 * control loop (Schedule / findNodesThatFit / prioritize / findBestNode /
 * Bind / Event) driving the GPU engine.
 *
 * Go is not installed in this image; a Go host would bind nas.h directly
 *  and keep its own loop.  This library is that loop in C++,
 * usable from C, C++, or Python (ctypes) with the cluster side supplied as
 * callbacks.  Same conventions as nas.h: int status returns, caller-owned
 * buffers, no exceptions across the ABI, a scheduler handle is not
 * thread-safe.
 */
#ifndef NAS_HOST_H_
#define NAS_HOST_H_

#include <stddef.h>
#include <stdint.h>

#include "nas.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the reference would have crashed (a Go runtime panic); message in the
 * panic buffer / nas_host_last_error */
#define NAS_HOST_PANIC (-10)

/* Go strconv error classes */
#define NAS_GO_OK 0
#define NAS_GO_ERR_SYNTAX 1
#define NAS_GO_ERR_RANGE 2

/* ---- stateless ingest (scheduler.go:396-549) ------------------------------ */

/* strconv.ParseFloat(s, bits): *value is Go's return value (also on error),
 * *go_err its error class. */
int nas_host_parse_float(const char *s, size_t n, int32_t bits, double *value, int32_t *go_err);
/* strconv.Atoi (64-bit int). */
int nas_host_atoi(const char *s, size_t n, int64_t *value, int32_t *go_err);

/* One node's record from its node-exporter text, in the struct-literal order
 * of :281-331 minus bandwidth: getCurrentCPUUsage (:409), getOccupiedMemory-
 * Percentage (:444), getNetworkPacketsReceived (:482), getNetworkPacketsSent
 * (:463), getDiskIONow (:532).  `node` selects the "ubuntu" or raspi
 * interface/disk names.  NAS_HOST_PANIC when a slice bound panics. */
int nas_host_node_metrics(const char *body, size_t n, const char *node, double *cpu, double *mem,
                          int64_t *rx, int64_t *tx, int64_t *disk, char *panic_msg,
                          size_t panic_cap);

/* A snapshot refresh: node i's node-exporter text bodies[i] (body_len[i]
 * bytes) under name names[i], each as nas_host_node_metrics, into SoA
 * arrays ready for nas_upload_snapshot (bandwidth comes from the iperf
 * reports, so the caller fills it).  status[i] = NAS_OK or NAS_HOST_PANIC
 * (that node's values are then 0: the reference would have crashed), or
 * NAS_ERR_STATE for a failure that is not a reference behaviour (e.g. out of
 * memory; values 0, and the call then returns NAS_ERR_STATE).  The
 * nodes are split over `threads` worker threads (<= 0: the hardware's
 * concurrency); the results do not depend on the thread count.  Replaces the
 * reference's per-pod sequential scrape-and-parse of :275-331 with one
 * parallel parse per refresh. */
int nas_host_snapshot_from_bodies(int32_t n, const char *const *bodies, const size_t *body_len,
                                  const char *const *names, double *cpu, double *mem, int64_t *rx,
                                  int64_t *tx, int64_t *disk, int32_t *status, int32_t threads);

/* json.Unmarshal into Iperf (:34-117, :551-555) and End.Streams[0]
 * (:525-528).  *n_streams == 0 is where the reference panics (index out of
 * range); *valid_json == 0 means Unmarshal rejected the document. */
int nas_host_iperf_receiver(const char *json, size_t n, double *receiver_bps, double *sender_bps,
                            int32_t *n_streams, int32_t *valid_json);

/* Pairwise latency (latency.h): reports[i*n+j] = iperf3 -J report of client
 * node i against server node j (NULL: none), lengths in report_len.  L_out
 * receives n*n int8 in ms per MB, symmetric, zero diagonal. */
int nas_host_latency_matrix(int32_t n, const char *const *reports, const size_t *report_len,
                            int8_t *L_out);
int32_t nas_host_latency_from_bps(double bps);
/* The unquantised form for NAS_DT_F32 placement: microseconds to move 1 MB
 * (8e12 / bps) as float, the slower direction of each pair, 0 on the
 * diagonal; a pair without a usable report costs 1e7 us (never Inf). */
int nas_host_latency_matrix_us(int32_t n, const char *const *reports, const size_t *report_len,
                               float *L_out);
float nas_host_latency_us_from_bps(double bps);

/* ---- the scheduler loop ----------------------------------------------------- */

typedef struct nas_host_buf nas_host_buf; /* output sink handed to callbacks */
void nas_host_buf_append(nas_host_buf *b, const char *data, size_t n);

/* The cluster side.  Callbacks return 0 on success; on failure they may put
 * a message in `err`. */
typedef struct nas_host_io {
    void *user;
    /* http.Get(url) + ReadAll (:396-407); nonzero: transport error (the
     * reference then dereferences a nil response: NAS_HOST_PANIC) */
    int (*http_get)(void *user, const char *url, nas_host_buf *body);
    /* os.Open + ReadAll of an iperf report (:512-520); nonzero: open failed */
    int (*read_file)(void *user, const char *path, nas_host_buf *bytes);
    /* nodeLister.List (:240): names separated by '\n' */
    int (*list_nodes)(void *user, nas_host_buf *names, nas_host_buf *err);
    /* Pods(ns).Bind (:196-206) */
    int (*bind)(void *user, const char *ns, const char *pod, const char *node, nas_host_buf *err);
    /* Events(ns).Create (:211-232) */
    int (*create_event)(void *user, const char *ns, const char *pod, const char *uid,
                        const char *message, nas_host_buf *err);
    /* network-aware path: a node's free capacity, and the node a pod
     * ("namespace/name") is bound to (empty: not bound) */
    int (*node_capacity)(void *user, const char *node, int32_t *cpu_milli, int32_t *mem_kib,
                         int32_t *pods);
    int (*pod_node)(void *user, const char *ns_name, nas_host_buf *node);
    /* Go map iteration orders for one prioritize call: order1[n] over the
     * scraped nodes, order2[n+1] over them plus "none" (= n) */
    void (*map_order)(void *user, int32_t n, int32_t *order1, int32_t *order2);
} nas_host_io;

typedef struct nas_host_sched nas_host_sched;

/* ctx: an engine context (nas_create) the scheduler uses; not owned. */
int nas_host_create(nas_host_sched **out, nas_ctx *ctx, const nas_host_io *io);
void nas_host_destroy(nas_host_sched *s);
const char *nas_host_last_error(nas_host_sched *s);

/* The scraped nodes (default: the reference's five, :275-279). */
int nas_host_set_topology(nas_host_sched *s, const char *const *names, const char *const *urls,
                          int32_t n);
/* Per-node iperf report paths, replacing the reference's map (:505-510). */
int nas_host_set_iperf_path(nas_host_sched *s, const char *node, const char *path);
/* Pairwise latency for the network-aware path, rows/cols named by names[]:
 * int8 ms (exact integer scores) or, _f32, measured microseconds (fp32 costs
 * on NAS_DT_F32; peer weights then enter as float MB).  The latency set last
 * decides the path of nas_host_place_pending. */
int nas_host_set_latency(nas_host_sched *s, const char *const *names, const int8_t *L, int32_t n);
int nas_host_set_latency_f32(nas_host_sched *s, const char *const *names, const float *L,
                             int32_t n);

typedef struct nas_host_pod {
    const char *ns, *name, *uid, *scheduler_name, *node_name;
    int32_t cpu_milli, mem_kib;       /* requests (network-aware path) */
    int32_t n_peers;
    const char *const *peers;         /* "namespace/name" of each peer pod */
    const int32_t *peer_weight;       /* traffic to each peer (any int32; exact sums) */
} nas_host_pod;

/* informer AddFunc (:166-176): 1 queued, 0 filtered out (bound, or another
 * scheduler), NAS_ERR_STATE when the 300-pod queue is full. */
int nas_host_enqueue(nas_host_sched *s, const nas_host_pod *p);
int32_t nas_host_queued(nas_host_sched *s);

#define NAS_HOST_BOUND 0
#define NAS_HOST_NO_POD 1
#define NAS_HOST_LIST_ERROR 2
#define NAS_HOST_BIND_ERROR 3
#define NAS_HOST_EVENT_ERROR 4
#define NAS_HOST_PANICKED 5
#define NAS_HOST_UNSCHEDULABLE 6

typedef struct nas_host_outcome {
    int32_t kind;       /* NAS_HOST_BOUND ... */
    char pod[128];      /* namespace/name */
    char node[128];     /* the node bound to (or tried) */
    char message[256];  /* event text, or the error / panic message */
} nas_host_outcome;

/* Schedule (:189-237): one pod. */
int nas_host_schedule_one(nas_host_sched *s, nas_host_outcome *out);
/* up to max_pods queued pods against one scrape, one GPU call. */
int nas_host_schedule_batch(nas_host_sched *s, int32_t max_pods, nas_host_outcome *out,
                            int32_t *n_out);
/* network-aware placement of every queued pod (nas_place); out holds
 * nas_host_queued() entries. */
int nas_host_place_pending(nas_host_sched *s, nas_host_outcome *out, int32_t *n_out);

#ifdef __cplusplus
}
#endif

#endif /* NAS_HOST_H_ */
