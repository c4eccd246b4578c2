"""Raw host->device copy bandwidth on the box (pinned and pageable sources,
one stream), the bound of every host-buffer call.  One JSON line per size."""
import json
import time

import torch


def main():
    dev = torch.device('cuda', 0)
    for mb in (16, 64, 360):
        n = mb << 20
        pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
        pageable = torch.empty(n, dtype=torch.uint8)
        pinned.fill_(1)
        pageable.fill_(1)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        out = {'mb': mb}
        for name, src in (('pinned', pinned), ('pageable', pageable)):
            d.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                d.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            out[name + '_GBps'] = round(n / min(ts) / 1e9, 1)
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
