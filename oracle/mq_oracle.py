"""CPU restatement of hyperdrive's MessageQueue (mq/mq.go), one message at a time.

TEST INFRASTRUCTURE ONLY: the checker of include/hd_mq.h in tests/; the
product never imports it.

  insert      mq.go:103-143  per-sender queue; sort.Search for the first
                             element with (height, round) greater than the
                             message's -> stable for equal keys; append + shift;
                             truncate to MaxCapacity (drops the largest)
  consume     mq.go:36-66    per sender, pop while height <= h; messages of
                             senders outside procsAllowed are dropped (not
                             delivered) but counted in n
  drop_below  mq.go:70-83    remove every message with height < h

Senders are the queue keys (the reference's map key is the message's From,
mq.go:107-113; any hashable here).  Sender iteration order: the reference walks
a Go map (unspecified order); this restatement, like the GPU queue, walks the
sender queues in the order they were created (a sender's first insert; the
map entry, and so its place, outlives an emptied queue, as in mq.go).
A message is any tuple whose [0] is height and [1] is round.
"""
from __future__ import annotations

import bisect
from typing import Dict, Hashable, List, Optional, Set, Tuple


class MessageQueue:
    def __init__(self, max_capacity: int = 1000):           # opt.go:19 default 1000
        self.max_capacity = max_capacity
        self.queues: Dict[Hashable, List[tuple]] = {}

    def insert(self, sender: Hashable, msg: tuple) -> None:
        q = self.queues.setdefault(sender, [])
        key = (msg[0], msg[1])
        # sort.Search: first index whose (height, round) > key  (mq.go:120-128)
        keys = [(m[0], m[1]) for m in q]
        at = bisect.bisect_right(keys, key)
        q.insert(at, msg)
        if len(q) > self.max_capacity:                       # mq.go:140-142
            del q[self.max_capacity:]

    def consume(self, h: int, allowed: Optional[Set[Hashable]] = None) -> Tuple[int, List[Tuple[Hashable, tuple]]]:
        n = 0
        out = []
        for sender in list(self.queues):                     # creation order (dicts keep insertion order)
            q = self.queues[sender]
            k = 0
            while k < len(q) and q[k][0] <= h:                # mq.go:38-41
                if allowed is None or sender in allowed:     # mq.go:49-51
                    out.append((sender, q[k]))
                n += 1
                k += 1
            self.queues[sender] = q[k:]
        return n, out

    def drop_below(self, h: int) -> None:
        for sender, q in self.queues.items():                # mq.go:70-83
            k = 0
            for m in q:
                if m[0] < h:
                    k += 1
            self.queues[sender] = q[k:]

    def __len__(self) -> int:
        return sum(len(q) for q in self.queues.values())
