"""Step time of the C2 all-pairs front-end under several extraction chunk schedules (one rendered scene).

    python tools/tune_frontend.py [images] "chunk,first" ...      e.g. "100,0" "50,0" "45,10" "25,0"
Prints one JSON line per schedule: host-to-host and device-resident ms per step and the stage split.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gtsfm_amd import native, synthetic  # noqa: E402
from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig  # noqa: E402


def timed(fe, steps, resident):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fe.step(resident=resident)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    n = int(sys.argv[1])
    dev = torch.device("cuda")
    native.lib()
    scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
    host = scene.images.cpu().pin_memory()
    del scene.images
    torch.cuda.empty_cache()
    for spec in sys.argv[2:]:
        ch, first = (int(x) for x in spec.split(","))
        fe = AllPairsFrontEnd(host, scene.intrinsics, n, 0, 1, dev, FrontEndConfig(extract_chunk=ch, extract_first=first))
        fe.step()
        fe.step()
        host_ms, res_ms = timed(fe, 5, False), timed(fe, 5, True)
        fe.instrument = True
        fe.step()
        torch.cuda.synchronize()
        st = {k: round(v, 3) for k, v in fe.stage_ms().items()}
        print(json.dumps({"chunk": ch, "first": first, "chunks": fe.chunks, "host_ms": round(host_ms, 3),
                          "resident_ms": round(res_ms, 3), "stage_ms": st}), flush=True)
        del fe
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
