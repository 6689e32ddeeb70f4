"""CPU: why the Map<K, Orswot> fold is not split over replica ranges (round 6).  Folding P consecutive
ranges and then the P partial states (a tree) gives a different state than the reference's left fold
`acc = Map::new(); for r: acc.merge(r)` (map.rs:140-220 with orswot.rs:81-183) on op-replay replicas:
a nested deferred remove survives the left fold and not the tree.  The GPU keeps the left fold (one
chain per key); the tree would have cut the config-4-scale causal fold from 11.4 to ~6.7 ms
(profiles/r06_mo_split.log)."""
import oracle as O


def test_map_orswot_tree_fold_differs_from_left_fold():
    R, K, M, A = 48, 4, 5, 4
    maps = O.map_orswot_objects(R, K, M, A, seed=81, steps=7 * R, p_vrm=0.5)
    left = O.map_fold_objects(maps)
    parts = [O.map_fold_objects(maps[j * 24:(j + 1) * 24]) for j in range(2)]
    tree = O.map_fold_objects(parts)
    assert tree.clock == left.clock and tree.deferred == left.deferred
    assert tree.entries != left.entries
    diff = [k for k in left.entries if tree.entries.get(k) != left.entries[k]]
    assert any(len(left.entries[k].val.deferred) > len(tree.entries[k].val.deferred) for k in diff if k in tree.entries)
