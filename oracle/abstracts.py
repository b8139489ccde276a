"""Index abstracts and the secondary-search join -- CPU restatement (TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product).

SURVEY.md §8f row 3.  A peer asked for a multi-word search answers with "index
abstracts": per include word, the url hashes of its container grouped by host
(WordReferenceFactory.compressIndex, WordReferenceFactory.java:75-117, built in
SearchEvent.java:505-531 and htroot/yacy/search.java:264-281).  The asking peer
decompresses them (decompressIndex :125-155, Protocol.java:576-596), merges
them per word (SecondarySearchSuperviser.addAbstract :43-65), joins the words
(SetTools.joinConstructive :76-200, SecondarySearchSuperviser.java:130) and
asks every peer that holds joined urls for exactly those urls and words
(prepareSecondarySearch :117-196, wordsFromPeer :71-87).

Strings are compared as Java Strings (UTF-16 code units, here ASCII bytes), so
TreeMap<String, ...> orders hosts, urls and peers by their raw bytes -- not by
Base64Order.  Parity is pinned by restatement (no reference fixture covers
these functions)."""

from typing import Dict, List, Optional, Sequence, Set, Tuple


def compress_index(container: Sequence[bytes], exclude: Optional[Sequence[bytes]] = None) -> bytes:
    """WordReferenceFactory.compressIndex(inputContainer, excludeContainer, maxtime)
    without its time limit: rows in container order; TreeMap<host, StringBuilder>."""
    ex = {bytes(r[:12]) for r in exclude} if exclude else set()
    doms: Dict[bytes, bytearray] = {}
    for r in container:
        u = bytes(r[:12])
        if u in ex:
            continue
        doms.setdefault(u[6:12], bytearray()).extend(u[0:6])
    parts = [h + b":" + bytes(doms[h]) for h in sorted(doms)]
    return b"{" + b",".join(parts) + b"}"


def decompress_index(ci: bytes, peerhash: bytes) -> Dict[bytes, Set[bytes]]:
    """WordReferenceFactory.decompressIndex (:125-155) for texts of the form
    compressIndex writes; url -> {peer}.  A text that is not of that form
    raises ValueError (the reference reads past the end of its buffer then)."""
    target: Dict[bytes, Set[bytes]] = {}
    if len(ci) < 2 or ci[0:1] != b"{" or ci[-1:] != b"}":
        return target
    ci = ci[1:-1]
    while len(ci) >= 13 and ci[6:7] == b":":
        dom = ci[0:6]
        ci = ci[7:]
        while ci and ci[0:1] != b",":
            if len(ci) < 6:
                raise ValueError("url run is not a multiple of 6 characters")
            url = ci[0:6] + dom
            ci = ci[6:]
            target.setdefault(url, set()).add(peerhash)
        if ci[0:1] == b",":
            ci = ci[1:]
    return target


class SecondarySearch:
    """SecondarySearchSuperviser: abstractsCache (TreeMap word -> url -> peers),
    addAbstract, prepareSecondarySearch."""

    def __init__(self):
        self.cache: Dict[bytes, Dict[bytes, Set[bytes]]] = {}
        self.checked: Set[bytes] = set()

    def add_abstract(self, word: bytes, single: Dict[bytes, Set[bytes]]) -> None:
        """addAbstract (:43-65): the first abstract of a word is stored as is; a
        later one puts each of its url -> peerlist entries into the stored map.
        put() returns the old set and the new peers are added to *that* set, which
        is no longer in the map: the map keeps the newest abstract's peer set."""
        old = self.cache.get(word)
        if old is None:
            self.cache[word] = single
            return
        for url, peers_new in single.items():
            peers_old = old.get(url)
            old[url] = peers_new
            if peers_old is not None:
                peers_old |= peers_new

    @staticmethod
    def join_constructive(maps: List[Dict[bytes, Set[bytes]]]) -> Dict[bytes, Set[bytes]]:
        """SetTools.joinConstructive(Collection, concatStrings=true) (:76-116):
        maps ordered by Long.valueOf(size * 1000 + count) (an int product, TreeMap
        put: an equal key replaces the earlier map), folded smallest first by
        joinConstructiveByTest; Set values are not Strings, so the running
        result's value is kept."""
        order: Dict[int, Dict[bytes, Set[bytes]]] = {}
        for count, m in enumerate(maps):
            if not m:
                return {}
            k = (len(m) * 1000 + count) & 0xFFFFFFFF
            if k >= 1 << 31:
                k -= 1 << 32
            order[k] = m
        if not order:
            return {}
        keys = sorted(order)
        res = order[keys[0]]
        for k in keys[1:]:
            if not res:
                break
            nxt = order[k]
            res = {u: v for u, v in res.items() if u in nxt}
        return dict(res)

    def prepare(self, include_words: Sequence[bytes], mypeer: bytes) -> Tuple[Dict[bytes, Set[bytes]],
                                                                           List[Tuple[bytes, List[bytes], List[bytes]]]]:
        """prepareSecondarySearch (:117-196) -> (abstractJoin, [(peer, urls, words)])
        for the peers asked, in peer order; urls and words sorted (they are
        HashSets in the reference; the request carries them as sets)."""
        if len(self.cache) != len(set(include_words)):
            return {}, []
        words = sorted(self.cache)
        join = self.join_constructive([self.cache[w] for w in words])
        if not join:
            return {}, []
        by_peer: Dict[bytes, Set[bytes]] = {}
        for url in sorted(join):
            for peer in join[url]:
                by_peer.setdefault(peer, set()).add(url)
        plan = []
        for peer in sorted(by_peer):
            if peer == mypeer or peer in self.checked:
                continue
            urls = by_peer[peer]
            ws = [w for w in words if any(peer in self.cache[w].get(u, ()) for u in urls)]
            if not ws:
                continue
            self.checked.add(peer)
            plan.append((peer, sorted(urls), ws))
        return join, plan
