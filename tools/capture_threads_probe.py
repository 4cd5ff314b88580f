"""Can a stream driven by a second host thread join a HIP graph capture begun by the first?
(tests/test_gpu_sharded_world2_distinct.py captures both ranks' bodies into one graph.)
Usage: python tools/capture_threads_probe.py MODE THREADED"""
import sys
import threading

import torch

mode, threaded = sys.argv[1], sys.argv[2] == "1"
dev = torch.device("cuda:0")
a = torch.arange(1 << 20, dtype=torch.float64, device=dev)
b = torch.zeros_like(a)
c = torch.zeros_like(a)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
box = {}
cv = threading.Condition()


def side():
    with cv:
        cv.wait_for(lambda: "start" in box)
        with torch.cuda.stream(s1):
            s1.wait_event(box["start"])
            c.copy_(a * 3)
            tmp = torch.empty_like(a)  # an allocation inside the capture, from this thread
            tmp.copy_(c + 1)
            c.copy_(tmp)
            e = torch.cuda.Event()
            e.record(s1)
            box["end"] = e
            cv.notify_all()


g = torch.cuda.CUDAGraph()
th = threading.Thread(target=side) if threaded else None
if th:
    th.start()
with torch.cuda.graph(g, stream=s0, capture_error_mode=mode):
    st = torch.cuda.Event()
    st.record(s0)
    if th:
        with cv:
            box["start"] = st
            cv.notify_all()
            cv.wait_for(lambda: "end" in box)
    else:
        box["start"] = st
        cv.acquire()
        cv.release()
        with torch.cuda.stream(s1):
            s1.wait_event(st)
            c.copy_(a * 3)
            tmp = torch.empty_like(a)
            tmp.copy_(c + 1)
            c.copy_(tmp)
            e = torch.cuda.Event()
            e.record(s1)
            box["end"] = e
    b.copy_(a * 2)
    s0.wait_event(box["end"])
if th:
    th.join()
g.replay()
torch.cuda.synchronize()
ok = torch.equal(b, a * 2) and torch.equal(c, a * 3 + 1)
print(f"mode={mode} threaded={threaded}: replay ok={ok}")
