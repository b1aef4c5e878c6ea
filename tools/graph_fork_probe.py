"""Does a captured side branch that forks a sub-branch and then waits on it
instantiate and replay as a hipGraph?  (The tower backward once put its
weight gradients on sub-branches of the candidate tower's branch; that
graph crashed at instantiation, so the sub-branches were joined from the
capture's origin stream instead.)

usage (GPU box): python tools/graph_fork_probe.py VARIANT
  origin_join  branch s1 forks s2; the ORIGIN stream joins s1 and s2
  nested_join  branch s1 forks s2 and joins it itself; the origin joins s1
  nested_twice as nested_join with two sub-branches forked from s1
Prints the step that fails (capture / instantiate / replay / values) or ok.
"""
import sys

import torch


def main(variant: str) -> None:
    dev = torch.device("cuda", 0)
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    out = {}

    def body():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        with torch.cuda.stream(s1):
            y = x * 2
            s2.wait_stream(s1)
            with torch.cuda.stream(s2):
                z = y + 1
            if variant == "nested_twice":
                s3.wait_stream(s1)
                with torch.cuda.stream(s3):
                    z2 = y + 2
            if variant in ("nested_join", "nested_twice"):
                s1.wait_stream(s2)  # the branch waits on the sub-branch it forked
                w = z * 3
                if variant == "nested_twice":
                    s1.wait_stream(s3)
                    w = w + z2
            else:
                w = y * 3
        cur.wait_stream(s1)
        if variant == "origin_join":
            cur.wait_stream(s2)
            w = w + z
        out["w"] = w

    body()  # eager warm-up (allocations)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    stage = "capture"

    def at(name):  # printed before the call, so a crash inside it is attributed
        print(f"{variant}: {name} ...", flush=True)
        return name

    try:
        with torch.cuda.stream(cap):
            stage = at("capture")
            g.capture_begin(capture_error_mode="thread_local")
            body()
            stage = at("capture_end (hipStreamEndCapture + hipGraphInstantiate)")
            g.capture_end()
        stage = at("replay")
        g.replay()
        torch.cuda.synchronize()
    except Exception as e:  # report which call failed
        print(f"{variant}: FAILED at {stage}: {e!r}")
        return
    if variant == "origin_join":
        ref = x * 2 * 3 + (x * 2 + 1)
    elif variant == "nested_join":
        ref = (x * 2 + 1) * 3
    else:
        ref = (x * 2 + 1) * 3 + (x * 2 + 2)
    print(f"{variant}: ok" if torch.equal(out["w"], ref) else f"{variant}: WRONG VALUES")


if __name__ == "__main__":
    main(sys.argv[1])
