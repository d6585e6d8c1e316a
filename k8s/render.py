#!/usr/bin/env python
"""Render Kubernetes manifests for a cluster of ps + worker tasks.

The reference's README claims a Kubernetes deployment but ships none; the inferred
contract is one pod per task, each running
``python /distributed_<m>.py --ps_hosts=... --worker_hosts=... --job_name=... --task_index=...``.
This renders exactly that: a headless Service per task (stable DNS name
``<name>-<job>-<i>``, port 2222) and a Job per task pinned to one MI355X
(``amd.com/gpu: 1``), the cluster spec built from those DNS names.

    python k8s/render.py --model gan --ps 1 --workers 2 --image dtfe-gan:latest > gan.yaml
    kubectl apply -f gan.yaml
"""
import argparse
import sys

PORT = 2222


def task_name(prefix, job, i):
    return "%s-%s-%d" % (prefix, job, i)


def render(model, n_ps, n_workers, image, prefix, gpus_per_task=1, extra=()):
    ps_hosts = ",".join("%s:%d" % (task_name(prefix, "ps", i), PORT) for i in range(n_ps))
    wk_hosts = ",".join("%s:%d" % (task_name(prefix, "worker", i), PORT) for i in range(n_workers))
    docs = []
    for job, n in (("ps", n_ps), ("worker", n_workers)):
        for i in range(n):
            name = task_name(prefix, job, i)
            labels = "app: %s\n    job: %s\n    task: \"%d\"" % (prefix, job, i)
            docs.append("""apiVersion: v1
kind: Service
metadata:
  name: %(name)s
spec:
  clusterIP: None
  selector:
    %(labels)s
  ports:
  - port: %(port)d
    targetPort: %(port)d""" % dict(name=name, labels=labels, port=PORT))
            args = ["--ps_hosts=" + ps_hosts, "--worker_hosts=" + wk_hosts, "--job_name=" + job,
                    "--task_index=%d" % i, "--workers=%d" % n_workers] + list(extra)
            docs.append("""apiVersion: batch/v1
kind: Job
metadata:
  name: %(name)s
spec:
  backoffLimit: 4          # restart a failed task; the chief restores from model_dir (SURVEY 5.3)
  template:
    metadata:
      labels:
        %(labels2)s
    spec:
      restartPolicy: OnFailure
      hostIPC: true
      containers:
      - name: %(job)s
        image: %(image)s
        args: [%(args)s]
        ports:
        - containerPort: %(port)d
        env:
        - {name: HSA_ENABLE_IPC_MODE_LEGACY, value: "0"}
        resources:
          limits: {amd.com/gpu: %(gpus)d}
        volumeMounts:
        - {name: ckpt, mountPath: /tmp/checkpoints}
      volumes:
      - name: ckpt
        emptyDir: {}""" % dict(name=name, labels2=labels.replace("\n    ", "\n        "), job=job, image=image,
                               args=", ".join('"%s"' % a for a in args), port=PORT, gpus=gpus_per_task))
    return "\n---\n".join(docs) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gan", choices=["gan", "encoder", "lstm", "softmax", "cnn"])
    ap.add_argument("--ps", type=int, default=1)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--image", default=None)
    ap.add_argument("--prefix", default=None)
    ap.add_argument("--gpus_per_task", type=int, default=1)
    ap.add_argument("extra", nargs=argparse.REMAINDER, help="extra flags passed to every task")
    a = ap.parse_args()
    sys.stdout.write(render(a.model, a.ps, a.workers, a.image or "dtfe-%s:latest" % a.model,
                            a.prefix or "dtfe-%s" % a.model, a.gpus_per_task, [x for x in a.extra if x != "--"]))


if __name__ == "__main__":
    main()
