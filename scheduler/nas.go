// cgo binding of the MI355X placement engine (include/nas.h) for the
// reference scheduler, scheduler/scheduler.go of pablojara/kubernetesNetAwareScheduler.
//
// This file goes next to scheduler.go (same `package main`).  The Go
// toolchain is not in the image this engine is built in, so it has not been
// compiled here; it uses only the C ABI that tests/test_abi.py checks symbol by
// symbol and that the C++ host mirror (kubernetesnetawarescheduler_amd/host/)
// drives the same way.  See INTEGRATION.md for the wiring.
//
// Replaced reference interfaces:
//   prioritize (scheduler.go:248-368) + findBestNode (:384-394), per pod
//       -> (*nasEngine).prioritizeAndPick            (nas_score_reference)
//   the same for a batch of pods sharing one scrape (:275-331)
//       -> (*nasEngine).prioritizeBatch               (nas_upload_pod_orders)
//   the network-aware placement decision of findNodesThatFit (:239-246)
//       -> (*nasEngine).placeBatch                    (nas_place)
//
// cgo rules kept: no Go pointer is retained by the library after a call
// returns (every entry is blocking and copies its inputs), and a nas_ctx is
// used from one OS thread per call (runtime.LockOSThread).

package main

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../kubernetesnetawarescheduler_amd -lnas -Wl,-rpath,${SRCDIR}/../kubernetesnetawarescheduler_amd
#include <stdlib.h>
#include "nas.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

type nasEngine struct {
	ctx   *C.nas_ctx
	names []string // node index <-> name, fixed at uploadNetwork / prioritize time
}

func nasErr(ctx *C.nas_ctx, rc C.int, what string) error {
	if rc == C.NAS_OK {
		return nil
	}
	return fmt.Errorf("%s: %s", what, C.GoString(C.nas_last_error(ctx)))
}

func newNasEngine(device int) (*nasEngine, error) {
	if v := int(C.nas_version()); v != int(C.NAS_ABI_VERSION) {
		return nil, fmt.Errorf("libnas ABI %d, header %d", v, int(C.NAS_ABI_VERSION))
	}
	var ctx *C.nas_ctx
	cfg := C.nas_config{device: C.int32_t(device)}
	if rc := C.nas_create(&ctx, &cfg); rc != C.NAS_OK {
		return nil, errors.New("nas_create failed (no GPU or libnas missing)")
	}
	// a peer rank that never arrives fails the call after 30 s instead of
	// blocking Schedule forever (NAS_OPT_COMM_TIMEOUT_MS)
	C.nas_set_option(ctx, C.NAS_OPT_COMM_TIMEOUT_MS, 30000)
	return &nasEngine{ctx: ctx}, nil
}

func (e *nasEngine) Close() {
	if e.ctx != nil {
		C.nas_destroy(e.ctx)
		e.ctx = nil
	}
}

// snapshot turns nodeMetricsMap (:281-331) into the SoA arrays of
// nas_upload_snapshot, node i = names[i].
func snapshot(names []string, metrics map[string]PrometheusNodeMetrics) (cpu, mem, bw []float64, rx, tx, disk []int64) {
	n := len(names)
	cpu, mem, bw = make([]float64, n), make([]float64, n), make([]float64, n)
	rx, tx, disk = make([]int64, n), make([]int64, n), make([]int64, n)
	for i, name := range names {
		m := metrics[name]
		cpu[i], mem[i], bw[i] = m.cpuFrequencyHertz, m.occupiedMemoryPercentage, m.networkBandwith
		rx[i], tx[i], disk[i] = int64(m.networkPacketsReceived), int64(m.networkPacketsSent), int64(m.diskIONow)
	}
	return
}

// mapOrders captures Go's iteration orders of the two maps the vote loop
// ranges over: `range nodeMetricsMap` (:334) and `range priorities` (:387,
// which also holds "none" = index n).  Passing them explicitly keeps the GPU
// result bit-identical to the Go loop's, ties included.
func mapOrders(names []string, metrics map[string]PrometheusNodeMetrics, priorities map[string]int) ([]int32, []int32) {
	n := len(names)
	idx := make(map[string]int32, n+1)
	for i, name := range names {
		idx[name] = int32(i)
	}
	idx["none"] = int32(n)
	order1 := make([]int32, 0, n)
	for name := range metrics {
		order1 = append(order1, idx[name])
	}
	order2 := make([]int32, 0, n+1)
	for name := range priorities {
		order2 = append(order2, idx[name])
	}
	return order1, order2
}

func (e *nasEngine) pick(best C.int32_t) string {
	switch best {
	case C.NAS_NONE:
		return "none" // the reference returns "none" too; Bind then fails (:207)
	case C.NAS_EMPTY:
		return ""
	}
	return e.names[int(best)]
}

func (e *nasEngine) uploadSnapshot(names []string, metrics map[string]PrometheusNodeMetrics) error {
	cpu, mem, bw, rx, tx, disk := snapshot(names, metrics)
	rc := C.nas_upload_snapshot(e.ctx, (*C.double)(&cpu[0]), (*C.double)(&mem[0]),
		(*C.int64_t)(&rx[0]), (*C.int64_t)(&tx[0]), (*C.double)(&bw[0]), (*C.int64_t)(&disk[0]),
		C.int32_t(len(names)), 1)
	e.names = names
	return nasErr(e.ctx, rc, "nas_upload_snapshot")
}

// prioritizeAndPick replaces prioritize + findBestNode (scheduler.go:248-394)
// for one pod, after the metric maps are filled (:281-331).
func (e *nasEngine) prioritizeAndPick(names []string, metrics map[string]PrometheusNodeMetrics,
	priorities map[string]int) (string, error) {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if err := e.uploadSnapshot(names, metrics); err != nil {
		return "", err
	}
	order1, order2 := mapOrders(names, metrics, priorities)
	var best C.int32_t
	if rc := C.nas_score_reference(e.ctx, (*C.int32_t)(&order1[0]), (*C.int32_t)(&order2[0]),
		nil, 1, &best, nil); rc != C.NAS_OK {
		return "", nasErr(e.ctx, rc, "nas_score_reference")
	}
	return e.pick(best), nil
}

// prioritizeBatch scores P queued pods against ONE scrape: one snapshot
// upload, and each pod's own map orders (its `priorities` map is built by
// the reference per call, :250-256, so its iteration order differs per pod).
func (e *nasEngine) prioritizeBatch(names []string, metrics map[string]PrometheusNodeMetrics,
	priorities []map[string]int) ([]string, error) {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	P, n := len(priorities), len(names)
	if P == 0 {
		return nil, nil
	}
	if err := e.uploadSnapshot(names, metrics); err != nil {
		return nil, err
	}
	order1 := make([]int32, 0, P*n)
	order2 := make([]int32, 0, P*(n+1))
	for _, pr := range priorities {
		o1, o2 := mapOrders(names, metrics, pr)
		order1 = append(order1, o1...)
		order2 = append(order2, o2...)
	}
	if rc := C.nas_upload_pod_orders(e.ctx, (*C.int32_t)(&order1[0]), (*C.int32_t)(&order2[0]),
		C.int32_t(P)); rc != C.NAS_OK {
		return nil, nasErr(e.ctx, rc, "nas_upload_pod_orders")
	}
	podSnap := make([]int32, P) // every pod on snapshot 0
	best := make([]int32, P)
	if rc := C.nas_score_reference(e.ctx, nil, nil, (*C.int32_t)(&podSnap[0]), C.int32_t(P),
		(*C.int32_t)(unsafe.Pointer(&best[0])), nil); rc != C.NAS_OK {
		return nil, nasErr(e.ctx, rc, "nas_score_reference")
	}
	out := make([]string, P)
	for p, b := range best {
		out[p] = e.pick(C.int32_t(b))
	}
	return out, nil
}

// uploadNetwork: the N x N latency matrix in microseconds (netperfScript /
// customNetworkBenchmark / clusterloader2 traces), fp32 as measured
// (NAS_DT_F32: no quantisation, costs within 1e-5 of fp64), and each node's
// free capacity.  Done once per netperf refresh / node-list change.
func (e *nasEngine) uploadNetwork(names []string, latencyUs []float32, cpuMilli, memKiB, pods []int32) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	n := len(names)
	if len(latencyUs) != n*n || len(cpuMilli) != n || len(memKiB) != n || len(pods) != n {
		return errors.New("uploadNetwork: sizes")
	}
	e.names = names
	if rc := C.nas_upload_latency(e.ctx, unsafe.Pointer(&latencyUs[0]), C.NAS_DT_F32, C.int32_t(n)); rc != C.NAS_OK {
		return nasErr(e.ctx, rc, "nas_upload_latency")
	}
	rc := C.nas_upload_capacity(e.ctx, (*C.int32_t)(&cpuMilli[0]), (*C.int32_t)(&memKiB[0]),
		(*C.int32_t)(&pods[0]), C.int32_t(n))
	return nasErr(e.ctx, rc, "nas_upload_capacity")
}

// placeBatch is the network-aware path: pods drained from podQueue (:129) in
// arrival order, each with its requests and its traffic (MB, fp32) to
// already-bound peers as CSR -- peerNode[rowPtr[p]:rowPtr[p+1]] is the node
// index of a bound peer or -1 -- are placed in one call.  The returned names
// are bound by the caller (bindPod, :370); "" means no node fits (requeue).
func (e *nasEngine) placeBatch(reqCPU, reqMemKiB, reqPods []int32, rowPtr, peerNode []int32,
	weightMB []float32) ([]string, error) {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	P := len(reqCPU)
	if P == 0 {
		return nil, nil
	}
	if len(reqMemKiB) != P || len(reqPods) != P || len(rowPtr) != P+1 ||
		len(peerNode) != len(weightMB) || int(rowPtr[P]) != len(peerNode) {
		return nil, errors.New("placeBatch: sizes")
	}
	if rc := C.nas_upload_pods(e.ctx, (*C.int32_t)(&reqCPU[0]), (*C.int32_t)(&reqMemKiB[0]),
		(*C.int32_t)(&reqPods[0]), C.int32_t(P)); rc != C.NAS_OK {
		return nil, nasErr(e.ctx, rc, "nas_upload_pods")
	}
	var peers *C.int32_t
	var weights unsafe.Pointer
	if len(peerNode) > 0 {
		peers, weights = (*C.int32_t)(&peerNode[0]), unsafe.Pointer(&weightMB[0])
	}
	if rc := C.nas_upload_traffic_csr(e.ctx, (*C.int32_t)(&rowPtr[0]), peers, weights, C.NAS_DT_F32,
		C.int32_t(P), C.int32_t(len(e.names)), C.int64_t(len(peerNode))); rc != C.NAS_OK {
		return nil, nasErr(e.ctx, rc, "nas_upload_traffic_csr")
	}
	node := make([]int32, P)
	if rc := C.nas_place(e.ctx, (*C.int32_t)(unsafe.Pointer(&node[0])), nil, nil); rc != C.NAS_OK {
		return nil, nasErr(e.ctx, rc, "nas_place")
	}
	out := make([]string, P)
	for p, b := range node {
		if b >= 0 {
			out[p] = e.names[b]
		}
	}
	return out, nil
}
