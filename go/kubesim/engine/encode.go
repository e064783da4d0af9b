package engine

/*
#include <stdlib.h>
#include "ks_engine.h"
#include "ks_ingest.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	"github.com/cpuguy83/strongerrors"
	"github.com/pkg/errors"
	"k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
)

// Resource order of the engine's arrays.
var resourceNames = [3]v1.ResourceName{v1.ResourceCPU, v1.ResourceMemory, "nvidia.com/gpu"}

const selImpossible = uint64(1) << 63 // a selector pair no node carries

// milli converts a quantity to the engine's int64 milli-units, refusing values that are not a
// whole number of milli-units or >= 2^59 (the exact domain, include/ks_engine.h).
func milli(q resource.Quantity) (int64, error) {
	m := q.MilliValue()
	if q.Cmp(*resource.NewMilliQuantity(m, q.Format)) != 0 || m < 0 || m >= 1<<59 {
		return 0, errors.Wrapf(ErrOutOfDomain, "quantity %s", q.String())
	}
	return m, nil
}

// Dicts are the taint and label dictionaries of a cluster: NoSchedule / NoExecute taints
// (the only effects the taint filter sees) and (key, value) labels, each mapped to a mask bit.
// Within one 64-bit mask every taint and pair has its own bit; a wider cluster encoded with
// NodeArraysFor shares bits between interchangeable taints and leaves unreferenced pairs out
// (include/ks_ingest.h ks_cluster_seal: the same rule as the C++ ingest).
type Dicts struct {
	taints    []v1.Taint
	taintBit  []int
	labels    map[[2]string]int
	nodePairs map[[2]string]bool
}

// NodeArrays encodes nodes (in config order: node index = tie-break order, kubesim.go:208-215)
// for Engine.LoadNodes and builds the dictionaries pods are encoded against; at most 64 distinct
// NoSchedule/NoExecute taints and 63 label pairs (use NodeArraysFor past that).
func NodeArrays(nodes []*v1.Node) (alloc []int64, taint, label []uint64, d *Dicts, err error) {
	return NodeArraysFor(nodes, nil)
}

// NodeArraysFor is NodeArrays for a cluster past one 64-bit mask, given every pod it will see
// (VERDICT r5 item 5): only the label pairs some pod's nodeSelector references get bits (no other
// label changes a placement: per-node hostname labels need none), and taints that exactly the same
// pods tolerate share one bit (a node is feasible for a pod iff the pod tolerates each of its
// taints).  With pods == nil, or a cluster within one mask, it is the plain encoding.
func NodeArraysFor(nodes []*v1.Node, pods []*v1.Pod) (alloc []int64, taint, label []uint64, d *Dicts, err error) {
	d = &Dicts{labels: map[[2]string]int{}, nodePairs: map[[2]string]bool{}}
	seen := map[[3]string]int{}
	alloc = make([]int64, 4*len(nodes))
	taint = make([]uint64, len(nodes))
	label = make([]uint64, len(nodes))
	nodeTaints := make([][]int, len(nodes))
	for i, n := range nodes {
		cap := n.Status.Capacity
		for k, name := range resourceNames {
			alloc[4*i+k] = -1
			if q, ok := cap[name]; ok {
				if alloc[4*i+k], err = milli(q); err != nil {
					return
				}
			}
		}
		alloc[4*i+3] = cap.Pods().Value() // absent => 0 (v1/resource.go:44-49)
		for _, t := range n.Spec.Taints {
			if t.Effect != v1.TaintEffectNoSchedule && t.Effect != v1.TaintEffectNoExecute {
				continue
			}
			key := [3]string{t.Key, t.Value, string(t.Effect)}
			b, ok := seen[key]
			if !ok {
				b = len(d.taints)
				seen[key] = b
				d.taints = append(d.taints, t)
			}
			nodeTaints[i] = append(nodeTaints[i], b)
		}
		for k, v := range n.ObjectMeta.Labels {
			d.nodePairs[[2]string{k, v}] = true
		}
	}
	// taint bits: one per taint, or one per class of equal toleration signatures over the pods
	d.taintBit = make([]int, len(d.taints))
	nbits := len(d.taints)
	if len(d.taints) > 64 && pods != nil {
		class := map[string]int{}
		for b := range d.taints {
			sig := make([]byte, len(pods))
			for j, pod := range pods {
				for i := range pod.Spec.Tolerations {
					if pod.Spec.Tolerations[i].ToleratesTaint(&d.taints[b]) {
						sig[j] = 1
						break
					}
				}
			}
			c, ok := class[string(sig)]
			if !ok {
				c = len(class)
				class[string(sig)] = c
			}
			d.taintBit[b] = c
		}
		nbits = len(class)
	} else {
		for b := range d.taints {
			d.taintBit[b] = b
		}
	}
	if nbits > 64 {
		return nil, nil, nil, nil, errors.Wrapf(ErrOutOfDomain, "%d distinct taint classes", nbits)
	}
	// label bits: every node pair, or the referenced ones past 63
	referenced := map[[2]string]bool{}
	for _, pod := range pods {
		for k, v := range pod.Spec.NodeSelector {
			referenced[[2]string{k, v}] = true
		}
	}
	wide := len(d.nodePairs) > 63 && pods != nil
	for i, n := range nodes {
		for k, v := range n.ObjectMeta.Labels {
			key := [2]string{k, v}
			if wide && !referenced[key] {
				continue
			}
			b, ok := d.labels[key]
			if !ok {
				if len(d.labels) == 63 {
					return nil, nil, nil, nil, errors.Wrap(ErrOutOfDomain, "more than 63 distinct (referenced) labels")
				}
				b = len(d.labels)
				d.labels[key] = b
			}
			label[i] |= 1 << uint(b)
		}
		for _, b := range nodeTaints[i] {
			taint[i] |= 1 << uint(d.taintBit[b])
		}
	}
	return alloc, taint, label, d, nil
}

// KeyTable interns pod keys "namespace-name" (kubesim/node/node.go:146-160) to int64 ids.
type KeyTable struct {
	ids map[string]int64
	bad int64
}

// ID of a pod's key; ok=false for an empty namespace or name (the pod fails at bind; it gets a
// fresh negative id so it never collides with another pod's key).
func (kt *KeyTable) ID(p *v1.Pod) (int64, bool) {
	if p.ObjectMeta.Namespace == "" || p.ObjectMeta.Name == "" {
		kt.bad--
		return kt.bad, false
	}
	if kt.ids == nil {
		kt.ids = map[string]int64{}
	}
	k := fmt.Sprintf("%s-%s", p.ObjectMeta.Namespace, p.ObjectMeta.Name)
	id, ok := kt.ids[k]
	if !ok {
		id = int64(len(kt.ids))
		kt.ids[k] = id
	}
	return id, true
}

// parseSimSpec parses a simSpec annotation in C (kubesim/pod/spec.go:25-63 rules, yaml.v2
// int32 decoding of `seconds`).  bad=true: the pod's bind fails with InvalidArgument.
func parseSimSpec(pod *v1.Pod) (sec []int32, use []int64, bad bool, err error) {
	annot, ok := pod.ObjectMeta.Annotations["simSpec"]
	if !ok {
		return nil, nil, true, nil // spec.go:27-29
	}
	ca := C.CString(annot)
	defer C.free(unsafe.Pointer(ca))
	var n C.int32_t
	const max = 256
	secs := make([]int32, max)
	usage := make([]int64, 3*max)
	mask := make([]uint8, max)
	var msg [256]C.char
	rc := C.ks_parse_simspec(ca, max, &n, (*C.int32_t)(unsafe.Pointer(&secs[0])),
		(*C.int64_t)(unsafe.Pointer(&usage[0])), (*C.uint8_t)(unsafe.Pointer(&mask[0])), &msg[0], 256)
	switch {
	case rc == C.KS_EINVAL:
		return nil, nil, true, nil
	case rc == C.KS_ERANGE:
		return nil, nil, false, errors.Wrap(ErrOutOfDomain, C.GoString(&msg[0]))
	case rc != C.KS_OK:
		return nil, nil, false, errors.Errorf("ks_parse_simspec: %d", int(rc))
	case int(n) > max:
		return nil, nil, false, errors.Wrapf(ErrOutOfDomain, "simSpec with %d phases", int(n))
	}
	return secs[:n], usage[:3*n], false, nil
}

// EncodePods turns pods returned by the submitters at tick `arrival` into the engine's records:
// requests summed over Spec.Containers (init containers and limits ignored,
// kubesim/node/resource.go:43-49), tolerations / nodeSelector as dictionary masks
// (toleration.go:37-56), the simSpec CSR, the key id.
func EncodePods(pods []*v1.Pod, arrival int64, d *Dicts, kt *KeyTable) (*Pods, error) {
	p := &Pods{PhaseOff: []int32{0}}
	for _, pod := range pods {
		var req [3]int64
		var km uint8
		for _, c := range pod.Spec.Containers {
			for k, name := range resourceNames {
				q, ok := c.Resources.Requests[name]
				if !ok {
					continue
				}
				m, err := milli(q)
				if err != nil {
					return nil, err
				}
				req[k] += m
				km |= 1 << uint(k)
			}
		}
		var tol, seen uint64
		for b := range d.taints {
			hit := false
			for i := range pod.Spec.Tolerations {
				if pod.Spec.Tolerations[i].ToleratesTaint(&d.taints[b]) {
					hit = true
					break
				}
			}
			bit := uint64(1) << uint(d.taintBit[b])
			if seen&bit != 0 && (tol&bit != 0) != hit { // a pod NodeArraysFor did not see splits a class
				return nil, errors.Wrap(ErrOutOfDomain, "a pod's tolerations split a taint class")
			}
			seen |= bit
			if hit {
				tol |= bit
			}
		}
		var sel uint64
		for k, v := range pod.Spec.NodeSelector {
			if b, ok := d.labels[[2]string{k, v}]; ok {
				sel |= 1 << uint(b)
			} else if d.nodePairs[[2]string{k, v}] { // a node pair NodeArraysFor saw unreferenced
				return nil, errors.Wrap(ErrOutOfDomain, "a nodeSelector pair without a mask bit")
			} else {
				sel |= selImpossible
			}
		}
		var flags uint8
		key, ok := kt.ID(pod)
		if !ok {
			flags |= C.KS_PODFLAG_BAD_KEY
		}
		sec, use, bad, err := parseSimSpec(pod)
		if err != nil {
			return nil, err
		}
		if bad {
			flags |= C.KS_PODFLAG_BAD_SPEC
		}
		p.Arrival = append(p.Arrival, arrival)
		p.Req = append(p.Req, req[:]...)
		p.KeyMask = append(p.KeyMask, km)
		p.Tol = append(p.Tol, tol)
		p.Sel = append(p.Sel, sel)
		p.PhaseSec = append(p.PhaseSec, sec...)
		p.PhaseUse = append(p.PhaseUse, use...)
		p.PhaseOff = append(p.PhaseOff, int32(len(p.PhaseSec)))
		p.Flags = append(p.Flags, flags)
		p.Key = append(p.Key, key)
	}
	if len(p.PhaseSec) > 1<<30 {
		return nil, strongerrors.InvalidArgument(errors.New("too many simSpec phases"))
	}
	return p, nil
}
