package engine

import (
	"context"
	"time"

	"github.com/pkg/errors"
	"k8s.io/api/core/v1"
	sched "k8s.io/kubernetes/pkg/scheduler/api"

	"github.com/ordovicia/kubernetes-simulator/api"
	"github.com/ordovicia/kubernetes-simulator/kubesim/clock"
	"github.com/ordovicia/kubernetes-simulator/kubesim/config"
)

// ErrPluginNotExpressible is returned by Run when a registered api.Filter / api.Scorer is not
// one of the device plugins (FitFilter, TaintFilter, SelectorFilter, ConstScorer,
// LeastRequestedScorer, BalancedAllocationScorer): the engine cannot call back into Go per
// (pod, node), and skipping the plugin silently would change results.  Use the reference's
// kubesim.KubeSim for such plugins.
var ErrPluginNotExpressible = errors.New("plugin cannot be evaluated on the device")

// KubeSim is kubesim.KubeSim (kubesim/kubesim.go:20-123) with the scheduling loop on the
// device: same constructor inputs, Register* methods and Run; one ks_step per tick.
type KubeSim struct {
	conf       *config.Config
	nodes      []*v1.Node
	nodeIndex  map[string]int32
	dicts      *Dicts
	keys       KeyTable
	submitters []api.Submitter
	filters    []api.Filter
	scorers    []api.Scorer
	device     int

	eng      *Engine
	base     int64              // FIFO index of pending[0]
	pending  []*v1.Pod          // submitted, not bound yet, FIFO order
	onBind   func(*v1.Pod, Bind) // optional observer (tests, metrics)
	tick     int64
	startClk clock.Clock
}

// NewKubeSim builds the simulated nodes from conf (config.BuildNode, in config order: the
// device's node index is the config position, which is the tie-break order).
func NewKubeSim(conf *config.Config, device int) (*KubeSim, error) {
	k := &KubeSim{conf: conf, nodeIndex: map[string]int32{}, device: device}
	for _, nc := range conf.Cluster.Nodes {
		n, err := config.BuildNode(nc, conf.StartClock)
		if err != nil {
			return nil, errors.Errorf("error building node config: %s", err.Error())
		}
		k.nodeIndex[n.Name] = int32(len(k.nodes))
		k.nodes = append(k.nodes, n)
	}
	return k, nil
}

// RegisterSubmitter registers a submitter plugin (kubesim/kubesim.go:73-76).
func (k *KubeSim) RegisterSubmitter(s api.Submitter) { k.submitters = append(k.submitters, s) }

// RegisterFilter registers a filter plugin (kubesim/kubesim.go:78-81); Run refuses plugins the
// device cannot evaluate (ErrPluginNotExpressible).
func (k *KubeSim) RegisterFilter(f api.Filter) { k.filters = append(k.filters, f) }

// RegisterScorer registers a scorer plugin (kubesim/kubesim.go:83-86).
func (k *KubeSim) RegisterScorer(s api.Scorer) { k.scorers = append(k.scorers, s) }

// OnBind sets an observer called for every bind, in FIFO order.
func (k *KubeSim) OnBind(f func(*v1.Pod, Bind)) { k.onBind = f }

// engineConfig maps the registered plugins onto ks_config.
func (k *KubeSim) engineConfig() (Config, error) {
	c := Config{TickSeconds: k.conf.Tick, Device: k.device}
	for _, f := range k.filters {
		switch f.(type) {
		case *FitFilter:
			c.Filters |= FilterFit
		case *TaintFilter:
			c.Filters |= FilterTaint
		case *SelectorFilter:
			c.Filters |= FilterSelector
		case *LiteralFilter, LiteralFilter:
			// the reference's own loop discards filter results (kubesim.go:182)
		default:
			return c, errors.Wrapf(ErrPluginNotExpressible, "filter %T", f)
		}
	}
	for _, s := range k.scorers {
		switch v := s.(type) {
		case *ConstScorer:
			c.Scorers = append(c.Scorers, ScorerSpec{ScorerConst, int32(v.Weight), int32(v.Value)})
		case ConstScorer:
			c.Scorers = append(c.Scorers, ScorerSpec{ScorerConst, int32(v.Weight), int32(v.Value)})
		case *LeastRequestedScorer:
			c.Scorers = append(c.Scorers, ScorerSpec{ScorerLeastRequested, int32(v.Weight), 0})
		case *BalancedAllocationScorer:
			c.Scorers = append(c.Scorers, ScorerSpec{ScorerBalanced, int32(v.Weight), 0})
		default:
			return c, errors.Wrapf(ErrPluginNotExpressible, "scorer %T", s)
		}
	}
	// FEEDS_SCORE once a filter that gates candidates is registered; the literal mode otherwise
	c.FeedsScore = c.Filters != 0 && !k.literal()
	return c, nil
}

func (k *KubeSim) literal() bool {
	for _, f := range k.filters {
		switch f.(type) {
		case *LiteralFilter, LiteralFilter:
			return true
		}
	}
	return false
}

// start creates the engine and loads the nodes (first Run).
func (k *KubeSim) start() error {
	if k.eng != nil {
		return nil
	}
	c, err := k.engineConfig()
	if err != nil {
		return err
	}
	alloc, taint, label, d, err := NodeArrays(k.nodes)
	if err != nil {
		return err
	}
	if k.eng, err = New(c); err != nil {
		return err
	}
	k.dicts = d
	return k.eng.LoadNodes(alloc, taint, label)
}

// Run executes the main loop (kubesim/kubesim.go:90-123): every tick the submitters are called
// in registration order, their pods are appended FIFO, and one queued pod is scheduled on the
// device; any plugin or CreatePod error ends the run with that error.
// The engine stays alive after Run returns (queries through Engine(), a later Run continues
// the same simulation); Close releases it, and so does the Engine's finalizer once the KubeSim is
// unreachable (a caller of the reference API, which has no Close, does not leak device memory).
func (k *KubeSim) Run(ctx context.Context) error {
	if err := k.start(); err != nil {
		return err
	}
	k.startClk = clock.NewClock(time.Now())
	nodes := k.nodes
	for {
		select {
		case <-ctx.Done():
			return ctx.Err()
		default:
		}
		k.tick++
		clk := k.startClk.Add(time.Duration(int64(k.conf.Tick)*k.tick) * time.Second)
		if err := k.submit(clk, nodes); err != nil {
			return err
		}
		if err := k.step(1); err != nil {
			return err
		}
	}
}

// PlacementBlind is implemented by an api.Submitter whose Submit never reads placement state —
// which pods are bound where, or usage — from its arguments (it may read the clock and the node
// list's static fields).  The reference example's submitter is one (examples/main.go:96-128).
type PlacementBlind interface {
	PlacementBlind() bool
}

// RunWindowed is Run for placement-blind submitters: each round calls the submitters for the
// next `window` ticks (clock and arrival tick exactly as Run would give them), then advances
// the device once over the whole window (one ks_step instead of `window`).  Binds, bind ticks
// and errors are identical to Run's — a pod's placement depends only on the pods submitted
// before it, and every submit happens before the step that binds it; a submitter error at tick t
// is returned after ticks < t are scheduled, as Run returns it.  ctx is checked once per window.
// One difference remains after an error: when the STEP fails at tick t (NotFound or
// InvalidArgument), the pods the submitters returned for ticks t+1 .. of the same window are
// already queued (Queued(), PodStatus report them Pending), whereas Run would never have called
// the submitters for those ticks.  Binds, ticks and the error itself are Run's.
// Every registered submitter must implement PlacementBlind (else an error, nothing run).
func (k *KubeSim) RunWindowed(ctx context.Context, window int64) error {
	if window <= 1 {
		return k.Run(ctx)
	}
	for _, s := range k.submitters {
		if b, ok := s.(PlacementBlind); !ok || !b.PlacementBlind() {
			return errors.New("RunWindowed: every submitter must implement PlacementBlind")
		}
	}
	if err := k.start(); err != nil {
		return err
	}
	k.startClk = clock.NewClock(time.Now())
	nodes := k.nodes
	for {
		select {
		case <-ctx.Done():
			return ctx.Err()
		default:
		}
		for i := int64(0); i < window; i++ {
			k.tick++
			clk := k.startClk.Add(time.Duration(int64(k.conf.Tick)*k.tick) * time.Second)
			if err := k.submit(clk, nodes); err != nil {
				if e2 := k.step(k.tick - 1 - k.eng.Tick()); e2 != nil {
					return e2
				}
				return err
			}
		}
		if err := k.step(k.tick - k.eng.Tick()); err != nil {
			return err
		}
	}
}

// Close releases the device engine (Run and RunWindowed leave it open for queries).
func (k *KubeSim) Close() {
	if k.eng != nil {
		k.eng.Close()
		k.eng = nil
	}
}

func (k *KubeSim) submit(clk clock.Clock, nodes []*v1.Node) error {
	for _, s := range k.submitters {
		pods, err := s.Submit(clk, nodes)
		if err != nil {
			return err
		}
		if len(pods) == 0 {
			continue
		}
		enc, err := EncodePods(pods, k.tick, k.dicts, &k.keys)
		if err != nil {
			return err
		}
		if err := k.eng.SubmitPods(enc); err != nil {
			return err
		}
		k.pending = append(k.pending, pods...)
	}
	return nil
}

// step runs `ticks` ticks on the device and writes each bind back into its v1.Pod
// (pod.Spec.NodeName, kubesim.go:222).  Binds carry global FIFO indices: pending holds the
// submitted-but-unbound pods from FIFO index base on.
func (k *KubeSim) step(ticks int64) error {
	binds, err := k.eng.Step(ticks)
	for _, b := range binds {
		pod := k.pending[b.Pod-k.base]
		pod.Spec.NodeName = k.nodes[b.Node].Name
		if k.onBind != nil {
			k.onBind(pod, b)
		}
	}
	if n := int64(len(binds)); n > 0 {
		last := binds[n-1].Pod
		k.pending = k.pending[last+1-k.base:]
		k.base = last + 1
	}
	return err
}

// Engine exposes the device engine (queries: UsageAt, PodLookup, NodePods, PodStatus).
func (k *KubeSim) Engine() *Engine { return k.eng }

// NodeIndex is a node's device index (config order).
func (k *KubeSim) NodeIndex(name string) (int32, bool) {
	i, ok := k.nodeIndex[name]
	return i, ok
}

// HostPriorities converts a device score row into the reference's HostPriorityList (hosts
// with no entry — score -1 — are left out, as nodeScore would leave them, kubesim.go:193-206).
func (k *KubeSim) HostPriorities(scores []int64) sched.HostPriorityList {
	var l sched.HostPriorityList
	for i, s := range scores {
		if s >= 0 {
			l = append(l, sched.HostPriority{Host: k.nodes[i].Name, Score: int(s)})
		}
	}
	return l
}
