"""Write tests/golden/reference_kats.json: the known-answer vectors held by the reference's
own unit tests, transcribed as data (inputs + expected outputs; quantities in milli-units):

  kubesim/util/util_test.go:13-41        BuildResourceList
  kubesim/pod/spec_test.go:16-77         parseSpecYAML (+ misspelled resourceUsagi ⇒ error)
  kubesim/node/resource_test.go:24-129   resourceListSum / Diff / GE
  kubesim/config/config_test.go:63-89    buildTaint effects (+ invalid effect ⇒ error)
  kubesim/clock/clock_test.go:35-48      Clock.Sub = 12h30m15s
  config/sample.yml:16-35 + examples/main.go:96-128  the C1 inputs as quantity strings
"""
import json, os
GI = 1 << 30
M = 1000
spec_ok = "\n- seconds: 5\n  resourceUsage:\n    cpu: 1\n    memory: 2Gi\n    nvidia.com/gpu: 0\n- seconds: 10\n  resourceUsage:\n    cpu: 2\n    memory: 4Gi\n    nvidia.com/gpu: 1\n"
kats = dict(
    build_resource_list=[
        dict(input={"cpu": "1", "memory": "2Gi", "nvidia.com/gpu": "1"},
             expect={"cpu": 1 * M, "memory": 2 * GI * M, "nvidia.com/gpu": 1 * M}),
        dict(input={"cpu": "1", "memory": "2Gi", "foo": "bar"}, expect="error"),
    ],
    parse_spec=[
        dict(input=spec_ok, expect=[[5, {"cpu": 1 * M, "memory": 2 * GI * M, "nvidia.com/gpu": 0}],
                                    [10, {"cpu": 2 * M, "memory": 4 * GI * M, "nvidia.com/gpu": 1 * M}]]),
        dict(input=spec_ok.replace("  resourceUsage:\n    cpu: 2", "  resourceUsagi:\n    cpu: 2"),
             expect="errInvalidResourceUsageField"),
    ],
    resource_list_sum=[
        dict(a={"cpu": 1 * M, "memory": 2 * GI * M}, b={"cpu": 2 * M, "memory": 4 * GI * M, "nvidia.com/gpu": 1 * M},
             expect={"cpu": 3 * M, "memory": 6 * GI * M, "nvidia.com/gpu": 1 * M}),
    ],
    resource_list_diff=[
        dict(a={"cpu": 2 * M, "memory": 4 * GI * M, "nvidia.com/gpu": 1 * M}, b={"cpu": 1 * M, "memory": 2 * GI * M},
             expect={"cpu": 1 * M, "memory": 2 * GI * M, "nvidia.com/gpu": 1 * M}),
        dict(a={"cpu": 1 * M, "memory": 2 * GI * M}, b={"cpu": 2 * M, "memory": 4 * GI * M, "nvidia.com/gpu": 1 * M},
             expect="errResourceListDiffNotGE"),
    ],
    resource_list_ge=[
        dict(a="r1", b="r1", expect=True), dict(a="r1", b="r2", expect=True), dict(a="r2", b="r1", expect=False),
        dict(a="r1", b="r3", expect=False), dict(a="r3", b="r1", expect=False),
    ],
    ge_lists=dict(r1={"cpu": 2 * M, "memory": 4 * GI * M, "nvidia.com/gpu": 1 * M},
                  r2={"cpu": 1 * M, "memory": 2 * GI * M},
                  r3={"cpu": 2 * M, "memory": 2 * GI * M, "nvidia.com/gpu": 2 * M}),
    build_taint=[dict(effect="NoSchedule", expect=1), dict(effect="NoExecute", expect=3),
                 dict(effect="PreferNoSchedule", expect=2), dict(effect="Invalid", expect="error")],
    clock_sub=dict(a="2018-01-01T12:30:15+09:00", b="2018-01-01T00:00:00+09:00", expect_seconds=12 * 3600 + 30 * 60 + 15),
    c1_inputs=dict(
        nodes=[{"cpu": "4", "memory": "8Gi", "nvidia.com/gpu": "1", "pods": "2"},
               {"cpu": "8", "memory": "16Gi", "nvidia.com/gpu": "2", "pods": "4"}],
        pod_requests={"cpu": "3", "memory": "5Gi", "nvidia.com/gpu": "1"},
        sim_spec=spec_ok, tick=10),
)
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json"), "w") as f:
    json.dump(kats, f, indent=1)
