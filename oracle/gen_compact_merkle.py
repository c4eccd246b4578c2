"""Golden (tree_size, hashes, root) states of the reference CompactMerkleTree
(ledger/compact_merkle_tree.py:13-193, with its MemoryHashStore and TreeHasher)
after a fixed sequence of append/extend calls over the leaves of
tests/golden/merkle.json.  Test infrastructure only: run here (the reference
is not on the GPU box), writes tests/golden/merkle_compact.json.

    python oracle/gen_compact_merkle.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(HERE, 'shims'), '/root/reference']

from ledger.compact_merkle_tree import CompactMerkleTree  # noqa: E402

STEPS = [1, 1, 3, 7, 16, 100, 5, 1, 300, 64, 2, 500]


def main():
    with open(os.path.join(REPO, 'tests', 'golden', 'merkle.json')) as fh:
        leaves = [bytes.fromhex(x) for x in json.load(fh)['leaves']]
    t, pos, states = CompactMerkleTree(), 0, []
    for k in STEPS:
        k = min(k, len(leaves) - pos)
        if k == 1:
            t.append(leaves[pos])
        else:
            t.extend(leaves[pos:pos + k])
        pos += k
        states.append({'extend': k, 'tree_size': t.tree_size, 'hashes': [h.hex() for h in t.hashes],
                       'root': t.root_hash.hex()})
    out = os.path.join(REPO, 'tests', 'golden', 'merkle_compact.json')
    with open(out, 'w') as fh:
        json.dump({'source': 'reference ledger.compact_merkle_tree.CompactMerkleTree, oracle/gen_compact_merkle.py',
                   'steps': states}, fh, indent=0)
    print('wrote', out, len(states), 'states, final size', pos)


if __name__ == '__main__':
    main()
