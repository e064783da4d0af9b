// The reference's example program (examples/main.go:43-69) on the device KubeSim: the same
// config, a submitter with the same output (one pod every 5 simulated seconds: requests cpu 3,
// memory 5Gi, gpu 1; simSpec 5 s {1, 2Gi, 0} then 10 s {2, 4Gi, 1}), and the always-true filter
// and constant scorer registered as their device forms.
package main

import (
	"context"
	"fmt"
	"os"
	"os/signal"
	"syscall"

	"github.com/pkg/errors"
	"github.com/spf13/viper"
	"k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"

	"github.com/ordovicia/kubernetes-simulator/kubesim/clock"
	"github.com/ordovicia/kubernetes-simulator/kubesim/config"
	"github.com/ordovicia/kubernetes-simulator/kubesim/engine"
	"github.com/ordovicia/kubernetes-simulator/log"
)

const spec = `
- seconds: 5
  resourceUsage: {cpu: "1", memory: 2Gi, nvidia.com/gpu: "0"}
- seconds: 10
  resourceUsage: {cpu: "2", memory: 4Gi, nvidia.com/gpu: "1"}
`

// everyFive submits pod-n once n*5 simulated seconds have passed since its first call.
type everyFive struct {
	start clock.Clock
	n     uint64
}

func (s *everyFive) Submit(c clock.Clock, _ []*v1.Node) ([]*v1.Pod, error) {
	if s.n == 0 {
		s.start = c
	}
	if uint64(c.Sub(s.start).Seconds())/5 < s.n {
		return nil, nil
	}
	req := v1.ResourceList{"cpu": resource.MustParse("3"), "memory": resource.MustParse("5Gi"),
		"nvidia.com/gpu": resource.MustParse("1")}
	p := &v1.Pod{
		ObjectMeta: metav1.ObjectMeta{Name: fmt.Sprintf("pod-%d", s.n), Namespace: "default",
			CreationTimestamp: c.ToMetaV1(), Annotations: map[string]string{"simSpec": spec}},
		Spec: v1.PodSpec{Containers: []v1.Container{{Name: "container", Image: "container",
			Resources: v1.ResourceRequirements{Requests: req}}}},
	}
	s.n++
	return []*v1.Pod{p}, nil
}

// PlacementBlind: Submit reads only the clock (engine.RunWindowed may call it ahead).
func (s *everyFive) PlacementBlind() bool { return true }

func readConfig(path string) (*config.Config, error) {
	viper.SetConfigName(path)
	viper.AddConfigPath(".")
	if err := viper.ReadInConfig(); err != nil {
		return nil, err
	}
	conf := config.Config{LogLevel: "info", Tick: 10, Cluster: config.ClusterConfig{Nodes: []config.NodeConfig{}}}
	return &conf, viper.Unmarshal(&conf)
}

func main() {
	ctx, cancel := context.WithCancel(context.Background())
	conf, err := readConfig("config/sample")
	if err != nil {
		log.L.Fatal(err)
	}
	k, err := engine.NewKubeSim(conf, 0)
	if err != nil {
		log.L.Fatal(err)
	}
	k.RegisterSubmitter(&everyFive{})
	k.RegisterFilter(engine.LiteralFilter{})                 // always true; results discarded
	k.RegisterScorer(engine.ConstScorer{Value: 1, Weight: 1}) // every node 1, weight 1
	sig := make(chan os.Signal, 1)
	signal.Notify(sig, syscall.SIGINT, syscall.SIGTERM)
	go func() {
		<-sig
		cancel()
	}()
	defer k.Close()
	// the submitter never reads placements: 1,024 ticks per device step, same binds as Run
	if err := k.RunWindowed(ctx, 1024); err != nil && errors.Cause(err) != context.Canceled {
		log.L.Fatal(err)
	}
}
