"""Deployment artefacts: per-task K8s manifests with the reference CLI, Dockerfiles."""
import os
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "k8s"))
import render  # noqa: E402


def test_render_one_pod_per_task_with_reference_cli():
    docs = list(yaml.safe_load_all(render.render("lstm", 2, 3, "img:1", "t")))
    assert len(docs) == 2 * (2 + 3)  # Service + Job per task
    jobs = [d for d in docs if d["kind"] == "Job"]
    args = {d["metadata"]["name"]: d["spec"]["template"]["spec"]["containers"][0]["args"] for d in jobs}
    a = args["t-worker-2"]
    assert "--ps_hosts=t-ps-0:2222,t-ps-1:2222" in a
    assert "--worker_hosts=t-worker-0:2222,t-worker-1:2222,t-worker-2:2222" in a
    assert "--job_name=worker" in a and "--task_index=2" in a and "--workers=3" in a
    svc = [d for d in docs if d["kind"] == "Service"]
    assert all(s["spec"]["clusterIP"] == "None" for s in svc)
    lim = jobs[0]["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert lim["amd.com/gpu"] == 1


def test_dockerfiles_present():
    assert os.path.exists(os.path.join(ROOT, "docker", "Dockerfile"))
    for m in ("gan", "encoder", "lstm"):
        txt = open(os.path.join(ROOT, "docker", m, "Dockerfile")).read()
        assert "distributed_%s.py" % m in txt
