// Package engine binds kubesim to the MI355X scheduling engine (libks_engine.so, C-ABI in
// include/ks_engine.h) through cgo.
//
// Placement in the reference: this directory is meant to sit at kubesim/engine/ of
// github.com/ordovicia/kubernetes-simulator, with include/ and the built libks_engine.so under
// third_party/ks/ (INTEGRATION.md).  It is written against the reference's interfaces
// (api/scheduler.go, api/submitter.go, kubesim/kubesim.go) and the header; neither this image
// nor the GPU box has a Go toolchain, so it has not been compiled here.
package engine

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/ks/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/ks/lib -lks_engine -Wl,-rpath,${SRCDIR}/../../third_party/ks/lib
#include <stdlib.h>
#include "ks_engine.h"
*/
import "C"

import (
	"runtime"
	"unsafe"

	"github.com/cpuguy83/strongerrors"
	"github.com/pkg/errors"
)

// ErrOutOfDomain: a valid input the engine refuses because it cannot keep results exact for it
// (KS_ERANGE: a quantity that is not a whole number of milli-units, a pod key reused while its
// earlier pod may still run, ...).  The caller may fall back to the reference's Go loop.
var ErrOutOfDomain = errors.New("outside the engine's exact domain")

// Engine is one simulated cluster on one device (a handle is single-threaded, like Run).
// n is the node count of LoadNodes: every per-node output buffer is sized from it, never from a
// caller's argument (the C side always writes n rows).
type Engine struct {
	h *C.ks_engine
	n int
}

func status(e *Engine, rc C.ks_status) error {
	msg := ""
	if e != nil && e.h != nil {
		msg = C.GoString(C.ks_last_error(e.h))
	}
	switch rc {
	case C.KS_OK:
		return nil
	case C.KS_ENOTFOUND: // kubesim/kubesim.go:217-220
		return strongerrors.NotFound(errors.New(msg))
	case C.KS_EINVAL:
		return strongerrors.InvalidArgument(errors.New(msg))
	case C.KS_ERANGE:
		return errors.Wrap(ErrOutOfDomain, msg)
	default:
		return errors.Errorf("ks_engine: device error (%d): %s", int(rc), msg)
	}
}

// Scorer kinds of ks_config (include/ks_engine.h).
const (
	ScorerConst          = C.KS_SCORER_CONST
	ScorerLeastRequested = C.KS_SCORER_LEAST_REQUESTED
	ScorerBalanced       = C.KS_SCORER_BALANCED
)

// Filter bits of ks_config.
const (
	FilterFit      = uint32(C.KS_FILTER_FIT)
	FilterTaint    = uint32(C.KS_FILTER_TAINT)
	FilterSelector = uint32(C.KS_FILTER_SELECTOR)
)

// Engine flags of ks_config (include/ks_engine.h): A/B and test switches; the defaults are the
// engine's choice.
const (
	FlagNoOverlap   = uint32(C.KS_ENGINE_NO_OVERLAP)   // the plain batch chain (no fused next-batch scan)
	FlagPrunedLists = uint32(C.KS_ENGINE_PRUNED_LISTS) // pruned block lists at any cluster size
)

// ScorerSpec is one registered device scorer (registration order is kept).
type ScorerSpec struct {
	Kind, Weight, Value int32
}

// Config of an engine.  FeedsScore=false reproduces the reference literally: its Filter result
// is discarded (kubesim/kubesim.go:182).
type Config struct {
	TickSeconds int
	FeedsScore  bool
	Filters     uint32
	Scorers     []ScorerSpec
	Device      int
	BatchPods   int
	EngineFlags uint32 // Flag* above (0: the engine's defaults)
}

func (c Config) toC() (C.ks_config, error) {
	var cfg C.ks_config
	if len(c.Scorers) > 8 {
		return cfg, strongerrors.InvalidArgument(errors.New("at most 8 scorers"))
	}
	cfg.abi_version = C.KS_ABI_VERSION
	cfg.tick_seconds = C.int32_t(c.TickSeconds)
	if c.FeedsScore {
		cfg.filter_mode = C.KS_FILTER_FEEDS_SCORE
	}
	cfg.filters = C.uint32_t(c.Filters)
	cfg.n_scorers = C.int32_t(len(c.Scorers))
	for i, s := range c.Scorers {
		cfg.scorers[i].kind = C.int32_t(s.Kind)
		cfg.scorers[i].weight = C.int32_t(s.Weight)
		cfg.scorers[i].value = C.int32_t(s.Value)
	}
	cfg.device = C.int32_t(c.Device)
	cfg.batch_pods = C.int32_t(c.BatchPods)
	cfg.engine_flags = C.uint32_t(c.EngineFlags)
	return cfg, nil
}

// New creates an engine (ks_create).
func New(c Config) (*Engine, error) {
	cfg, err := c.toC()
	if err != nil {
		return nil, err
	}
	e := &Engine{}
	if rc := C.ks_create(&cfg, &e.h); rc != C.KS_OK {
		return nil, errors.Errorf("ks_create rejected the configuration (%d)", int(rc))
	}
	// A caller written against the reference API never calls Close (kubesim.KubeSim has none):
	// the device state is released when the Engine becomes unreachable.
	runtime.SetFinalizer(e, (*Engine).Close)
	return e, nil
}

// Close releases the device state.
func (e *Engine) Close() {
	if e.h != nil {
		C.ks_destroy(e.h)
		e.h = nil
	}
	runtime.SetFinalizer(e, nil)
}

// CommUniqueID makes the RCCL communicator id rank 0 broadcasts to the others (ks_comm_unique_id).
func CommUniqueID() ([]byte, error) {
	id := make([]byte, C.KS_COMM_ID_BYTES)
	if rc := C.ks_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&id[0]))); rc != C.KS_OK {
		return nil, status(nil, rc)
	}
	return id, nil
}

// Shard makes this engine rank `rank` of `world` node-sharded engines (one per GPU, ks_shard):
// each scans its node range and the per-pod candidate lists are all-gathered over RCCL once per
// batch; every rank loads the whole cluster and submits the same pods, and all binds are
// identical.  Call before LoadNodes.
func (e *Engine) Shard(world, rank int, id []byte, vshards int) error {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	if len(id) != C.KS_COMM_ID_BYTES {
		return errors.Errorf("communicator id: %d bytes, want %d", len(id), C.KS_COMM_ID_BYTES)
	}
	rc := C.ks_shard(e.h, C.int32_t(world), C.int32_t(rank), (*C.uint8_t)(unsafe.Pointer(&id[0])), C.int32_t(vshards))
	return status(e, rc)
}

// LoadNodes loads the cluster once: alloc = n*4 {milli cpu, milli memory, milli gpu, pods}
// (-1 = key absent), taint / label = dictionary bitmasks (Dicts).
func (e *Engine) LoadNodes(alloc []int64, taint, label []uint64) error {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	n := len(taint)
	if len(alloc) != 4*n || len(label) != n {
		return strongerrors.InvalidArgument(errors.New("LoadNodes: alloc must hold 4 values per node"))
	}
	if n == 0 {
		return status(e, C.ks_load_nodes(e.h, 0, nil, nil, nil))
	}
	err := status(e, C.ks_load_nodes(e.h, C.int64_t(n), (*C.int64_t)(unsafe.Pointer(&alloc[0])),
		(*C.uint64_t)(unsafe.Pointer(&taint[0])), (*C.uint64_t)(unsafe.Pointer(&label[0]))))
	if err == nil {
		e.n = n
	}
	return err
}

// Pods is a batch of encoded pods in FIFO order (EncodePods builds it from []*v1.Pod).
type Pods struct {
	Arrival  []int64 // the tick whose Submit returned the pod
	Req      []int64 // 3 per pod, milli-units
	KeyMask  []uint8 // request keys present: 1 cpu, 2 memory, 4 gpu
	Tol, Sel []uint64
	PhaseOff []int32 // len(Arrival)+1
	PhaseSec []int32
	PhaseUse []int64 // 3 per phase
	Flags    []uint8 // KS_PODFLAG_*
	Key      []int64 // interned "namespace-name" (KeyTable)
}

func i64p(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}
func u64p(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}
func i32p(s []int32) *C.int32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int32_t)(unsafe.Pointer(&s[0]))
}
func u8p(s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}

// SubmitPods appends pods to the FIFO (submit + podQueue.append, kubesim/kubesim.go:126-139).
func (e *Engine) SubmitPods(p *Pods) error {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	m := len(p.Arrival)
	if m == 0 {
		return nil
	}
	if len(p.Req) != 3*m || len(p.KeyMask) != m || len(p.Tol) != m || len(p.Sel) != m ||
		len(p.PhaseOff) != m+1 || len(p.Flags) != m || len(p.Key) != m ||
		int(p.PhaseOff[m]) > len(p.PhaseSec) || 3*int(p.PhaseOff[m]) > len(p.PhaseUse) {
		return strongerrors.InvalidArgument(errors.New("SubmitPods: inconsistent array lengths"))
	}
	return status(e, C.ks_submit_pods(e.h, C.int64_t(m), i64p(p.Arrival), i64p(p.Req), u8p(p.KeyMask),
		u64p(p.Tol), u64p(p.Sel), i32p(p.PhaseOff), i32p(p.PhaseSec), i64p(p.PhaseUse), u8p(p.Flags),
		i64p(p.Key)))
}

// Bind is one scheduling decision: FIFO index, node index, status (0 Ok, 1 OverCapacity,
// kubesim/pod/pod.go:20-27) and bind tick.
type Bind struct {
	Pod    int64
	Node   int32
	Status int32
	Tick   int64
}

// Queued is the number of submitted pods not popped yet.
func (e *Engine) Queued() int64 {
	defer runtime.KeepAlive(e)
	return int64(C.ks_queued_pods(e.h))
}

// Tick is the engine's current tick.
func (e *Engine) Tick() int64 {
	defer runtime.KeepAlive(e)
	return int64(C.ks_current_tick(e.h))
}

// TickSeconds is the simulated seconds per tick (ks_tick_seconds): the submitters' clock is
// start + Tick() * TickSeconds().
func (e *Engine) TickSeconds() int64 {
	defer runtime.KeepAlive(e)
	return int64(C.ks_tick_seconds(e.h))
}

// Step advances `ticks` ticks of Run's loop (at most one bind per tick).  Binds made before an
// aborting error (NotFound / InvalidArgument) are returned with the error.
func (e *Engine) Step(ticks int64) ([]Bind, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	cap := ticks
	if q := e.Queued(); q < cap {
		cap = q
	}
	if cap < 0 {
		cap = 0
	}
	out := make([]C.ks_bind, cap+1)
	var n C.int64_t
	rc := C.ks_step(e.h, C.int64_t(ticks), &out[0], C.int64_t(cap), &n)
	k := int64(n)
	if k > cap {
		k = cap
	}
	binds := make([]Bind, k)
	for i := range binds {
		binds[i] = Bind{int64(out[i].pod), int32(out[i].node), int32(out[i].status), int64(out[i].tick)}
	}
	return binds, status(e, rc)
}

// FilterMask is api.Filter over every node for queued pod `pod` (ks_filter): one byte per
// loaded node.
func (e *Engine) FilterMask(pod int64) ([]uint8, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	mask := make([]uint8, e.n+1)
	return mask[:e.n], status(e, C.ks_filter(e.h, C.int64_t(pod), u8p(mask)))
}

// Scores is the aggregated score of every loaded node for queued pod `pod` (-1 = no entry,
// ks_score).
func (e *Engine) Scores(pod int64) ([]int64, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	s := make([]int64, e.n+1)
	return s[:e.n], status(e, C.ks_score(e.h, C.int64_t(pod), i64p(s)))
}

// UsageAt is Σ Pod.ResourceUsage per node at tick t <= Tick() (3 per loaded node: cpu, memory,
// gpu milli).
func (e *Engine) UsageAt(t int64) ([]int64, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	u := make([]int64, 3*e.n+1)
	return u[:3*e.n], status(e, C.ks_usage_at(e.h, C.int64_t(t), i64p(u)))
}

// Nodes is the node count of LoadNodes.
func (e *Engine) Nodes() int { return e.n }

// PodLookup is Node.GetPod by key (kubesim/node/node.go:62-75): the FIFO index stored there.
func (e *Engine) PodLookup(node int32, key int64) (int64, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	var q C.int64_t
	err := status(e, C.ks_pod_lookup(e.h, C.int32_t(node), C.int64_t(key), &q))
	return int64(q), err
}

// NodePods is Node.GetPodList (kubesim/node/node.go:77-82): FIFO indices, one per key.
func (e *Engine) NodePods(node int32) ([]int64, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	var n C.int64_t
	if err := status(e, C.ks_node_pods(e.h, C.int32_t(node), nil, 0, &n)); err != nil {
		return nil, err
	}
	out := make([]int64, int(n)+1)
	err := status(e, C.ks_node_pods(e.h, C.int32_t(node), i64p(out), n, &n))
	return out[:int(n)], err
}

// PodPhase values of ks_pod_info.
const (
	PhasePending   = C.KS_PHASE_PENDING
	PhaseRunning   = C.KS_PHASE_RUNNING
	PhaseSucceeded = C.KS_PHASE_SUCCEEDED
	PhaseFailed    = C.KS_PHASE_FAILED
)

// PodInfo is Pod.BuildStatus's data (kubesim/pod/pod.go:78-167) at the current tick.
type PodInfo struct {
	Phase        int32
	Node         int32
	StartTick    int64
	TotalSeconds int32
}

// PodStatus returns the status of FIFO pods [lo, lo+n).
func (e *Engine) PodStatus(lo, n int64) ([]PodInfo, error) {
	defer runtime.KeepAlive(e) // e.h must outlive the C call (the finalizer runs ks_destroy)
	out := make([]C.ks_pod_info, n+1)
	if err := status(e, C.ks_pod_status(e.h, C.int64_t(lo), C.int64_t(n), &out[0])); err != nil {
		return nil, err
	}
	r := make([]PodInfo, n)
	for i := range r {
		r[i] = PodInfo{int32(out[i].phase), int32(out[i].node), int64(out[i].start_tick), int32(out[i].total_seconds)}
	}
	return r, nil
}
