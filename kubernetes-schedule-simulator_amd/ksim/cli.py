"""k8s-scheduler-simulator's command line over the HIP path.

    python -m ksim.cli --podspec etc/pod.yaml --nodes nodes.json [--pods pods.json]
                       [--algorithmprovider DefaultProvider | --policy-config-file policy.json]
                       [--namespace NS] [--uuid-names] [--json]

Reference: cmd/app/server.go:40-110 (flags from cmd/app/options/options.go:64-69, podspec parsing
:73-99, run + ClusterCapacityReviewPrint) and the offline checkpoint path of pkg/main.go:134-179
(nodes.json / pods.json arrays of v1.Node / v1.Pod).  The snapshot comes from the checkpoint
files: listing a live cluster through --kubeconfig needs an API server and is out of scope
(SURVEY.md §8), so that flag is refused rather than ignored.  Pods in pods.json are the
already-running pods (getCheckpoints lists status.phase=Running; here the file is taken as it
is, like anaCheckPoint).  Exit status 1 with a message on every error, like glog.Fatalf.
"""
from __future__ import annotations

import argparse
import json
import sys


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="k8s-scheduler-simulator",
                                 description="Simulate kube-scheduler placement of a pod spec on a cluster snapshot (MI355X).")
    ap.add_argument("--podspec", required=True, help="Path to JSON or YAML file containing pod definition.")
    ap.add_argument("--nodes", required=True, help="nodes.json checkpoint: JSON array of v1.Node.")
    ap.add_argument("--pods", default=None, help="pods.json checkpoint: JSON array of running v1.Pod.")
    ap.add_argument("--algorithmprovider", default="DefaultProvider", help="Kubernetes scheduler algorithm provider.")
    ap.add_argument("--policy-config-file", default=None, help="Scheduler Policy file (overrides the provider).")
    ap.add_argument("--namespace", default="", help="Namespace given to the simulation pods.")
    ap.add_argument("--kubeconfig", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--uuid-names", action="store_true", help="Name simulation pods with uuid4s as the reference does.")
    ap.add_argument("--json", action="store_true", help="Print GetReport's review as JSON instead of the tables.")
    ap.add_argument("--device", type=int, default=0)
    return ap.parse_args(argv)


def _json_default(o):
    return str(o)


def main(argv=None) -> int:
    a = parse_args(argv)
    from . import scheduler
    from .report import review_text
    if a.kubeconfig:
        print("--kubeconfig: listing a live cluster is not supported; pass --nodes/--pods checkpoint files",
              file=sys.stderr)
        return 1
    try:
        spec = scheduler.load_podspec(a.podspec)
        sim = scheduler.expand_simulation_pods(spec or [], a.namespace, uid="uuid" if a.uuid_names else None)
        nodes, running = scheduler.load_checkpoint(a.nodes, a.pods)
        pol = None
        if a.policy_config_file:
            from . import policy
            pol = policy.load(a.policy_config_file)
        cc = scheduler.ClusterCapacity(nodes, running, sim, provider_name=a.algorithmprovider, policy_obj=pol,
                                       device=a.device)
        rep = cc.run()
    except Exception as e:  # glog.Fatalf("Failed to start scheduler simulator: %v", err)
        print("Failed to start scheduler simulator: %s" % e, file=sys.stderr)
        return 1
    if a.json:
        print(json.dumps(rep.review, default=_json_default, indent=1))
    else:
        sys.stdout.write(review_text(rep.review))
    return 0


if __name__ == "__main__":
    sys.exit(main())
