"""The ``checkpoint`` state file (text-format ``CheckpointState`` proto).

    model_checkpoint_path: "model.ckpt-200"
    all_model_checkpoint_paths: "model.ckpt-100"
    all_model_checkpoint_paths: "model.ckpt-200"
"""
import os
import re

STATE_FILE = "checkpoint"


def _q(s):
    return '"%s"' % s.replace("\\", "\\\\").replace('"', '\\"')


def write_state(directory, model_checkpoint_path, all_paths):
    # TF convention: paths are stored relative to the save directory, whether the caller passed
    # them relative to the working directory ("ck/model.ckpt-1") or absolute.
    base = os.path.abspath(directory)

    def rel(p):
        return os.path.relpath(os.path.abspath(p), base)
    lines = ["model_checkpoint_path: %s" % _q(rel(model_checkpoint_path))]
    lines += ["all_model_checkpoint_paths: %s" % _q(rel(p)) for p in all_paths]
    tmp = os.path.join(directory, STATE_FILE + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(directory, STATE_FILE))


def read_state(directory):
    path = os.path.join(directory, STATE_FILE)
    if not os.path.exists(path):
        return None
    model, all_paths = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).replace('\\"', '"').replace("\\\\", "\\")
            if not os.path.isabs(v):
                v = os.path.join(directory, v)
            if k == "model_checkpoint_path":
                model = v
            elif k == "all_model_checkpoint_paths":
                all_paths.append(v)
    return {"model_checkpoint_path": model, "all_model_checkpoint_paths": all_paths}


def latest_checkpoint(directory):
    if not directory or not os.path.isdir(directory):
        return None
    st = read_state(directory)
    if st and st["model_checkpoint_path"] and os.path.exists(st["model_checkpoint_path"] + ".index"):
        return st["model_checkpoint_path"]
    return None
