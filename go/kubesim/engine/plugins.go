package engine

import (
	"github.com/pkg/errors"
	"k8s.io/api/core/v1"
	sched "k8s.io/kubernetes/pkg/scheduler/api"
)

// Device plugins: registering these on a KubeSim selects the engine's built-in predicates and
// scorers (ks_config).  They also satisfy api.Filter / api.Scorer, so they can be registered on
// the reference's own kubesim.KubeSim — there they answer through a device Engine attached with
// Attach (ks_filter / ks_score on the pod's FIFO index), or fail with ErrNoEngine.

// ErrNoEngine: a device plugin was called with no engine attached.
var ErrNoEngine = errors.New("device plugin has no engine attached")

// FitFilter is Node.CreatePod's admission test as a Filter (kubesim/node/node.go:44-47).
type FitFilter struct{ Device }

// TaintFilter passes nodes whose NoSchedule / NoExecute taints the pod tolerates
// (vendor/k8s.io/api/core/v1/toleration.go:37-56).
type TaintFilter struct{ Device }

// SelectorFilter passes nodes carrying every nodeSelector pair of the pod.
type SelectorFilter struct{ Device }

// LiteralFilter is examples/main.go's always-true filter (kubesim.go:182 discards filter
// results anyway): registering it keeps the engine in the reference-literal mode.
type LiteralFilter struct{}

// Filter implements api.Filter (examples/main.go:142-144).
func (LiteralFilter) Filter(pod *v1.Pod, node *v1.Node) (bool, error) { return true, nil }

// ConstScorer gives every node Value (examples/main.go:147-155 is Value 1, Weight 1).
type ConstScorer struct {
	Value, Weight int
}

// Score implements api.Scorer.
func (s ConstScorer) Score(pod *v1.Pod, nodes []*v1.Node) (sched.HostPriorityList, int, error) {
	l := make(sched.HostPriorityList, 0, len(nodes))
	for _, n := range nodes {
		l = append(l, sched.HostPriority{Host: n.Name, Score: s.Value})
	}
	return l, s.Weight, nil
}

// LeastRequestedScorer: (A - u) * 10 / A averaged over cpu and memory, integer (SURVEY §8 a14).
type LeastRequestedScorer struct {
	Weight int
	Device
}

// BalancedAllocationScorer: floor(10 (1 - |u_c/A_c - u_m/A_m|)), exact integer form.
type BalancedAllocationScorer struct {
	Weight int
	Device
}

// Device attaches a plugin to an engine for use inside the reference's own loop: the pod is
// found in the engine's FIFO by its key (the caller submitted it with the same KeyTable).
type Device struct {
	k *KubeSim
}

// Attach binds the plugin to a device KubeSim.
func (d *Device) Attach(k *KubeSim) { d.k = k }

func (d *Device) fifoIndex(pod *v1.Pod) (int64, error) {
	if d.k == nil || d.k.eng == nil {
		return 0, ErrNoEngine
	}
	for i, p := range d.k.pending {
		if p == pod {
			return d.k.base + int64(i), nil
		}
	}
	return 0, errors.Errorf("pod %s/%s is not queued on the engine", pod.Namespace, pod.Name)
}

// Filter implements api.Filter over ks_filter (every enabled device filter of the engine).
func (d *Device) Filter(pod *v1.Pod, node *v1.Node) (bool, error) {
	q, err := d.fifoIndex(pod)
	if err != nil {
		return false, err
	}
	i, ok := d.k.NodeIndex(node.Name)
	if !ok {
		return false, errors.Errorf("node %q unknown to the engine", node.Name)
	}
	mask, err := d.k.eng.FilterMask(q)
	if err != nil {
		return false, err
	}
	return mask[i] != 0, nil
}

// Score implements api.Scorer over ks_score: the engine's aggregated score (all registered
// device scorers, weights applied), returned with weight 1 for the requested nodes.
func (d *Device) Score(pod *v1.Pod, nodes []*v1.Node) (sched.HostPriorityList, int, error) {
	q, err := d.fifoIndex(pod)
	if err != nil {
		return nil, 0, err
	}
	all, err := d.k.eng.Scores(q)
	if err != nil {
		return nil, 0, err
	}
	l := make(sched.HostPriorityList, 0, len(nodes))
	for _, n := range nodes {
		if i, ok := d.k.NodeIndex(n.Name); ok && all[i] >= 0 {
			l = append(l, sched.HostPriority{Host: n.Name, Score: int(all[i])})
		}
	}
	return l, 1, nil
}
