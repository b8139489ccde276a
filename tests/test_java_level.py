"""The Java drop-in (java/) stays within Java 8, YaCy's own language level.

YaCy compiles with -source 1.8 -target 1.8 (/root/reference/build.properties:2-3,
pom.xml:34-35) and its CI runs oraclejdk8 (.travis.yml:8-9).  The image has no
JDK, so the drop-in cannot be compiled here; this test scans its sources (comments
and string literals removed) for language features and library APIs that arrived
after Java 8, and fails on any hit.  The scanner is checked against snippets that
must be caught and snippets that must pass."""

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java")

# (pattern, what it is, the Java version that added it)
POST_JAVA8 = [
    (r"\bjava\.lang\.ref\.Cleaner\b|\bCleaner\s*\.\s*(create|Cleanable)\b", "java.lang.ref.Cleaner", 9),
    (r"\b(List|Set|Map)\s*\.\s*(of|copyOf|ofEntries)\s*\(", "immutable collection factories", 9),
    (r"\bMap\s*\.\s*entry\s*\(", "Map.entry", 9),
    (r"(^|[;{}(\s])var\s+[A-Za-z_]\w*\s*[=:]", "local variable type inference (var)", 10),
    (r"\.\s*orElseThrow\s*\(\s*\)", "Optional.orElseThrow()", 10),
    (r"\.\s*(strip|stripLeading|stripTrailing|isBlank)\s*\(\s*\)", "String.strip / isBlank", 11),
    (r"\.\s*repeat\s*\(", "String.repeat", 11),
    (r"\.\s*readAllBytes\s*\(\s*\)|\.\s*readNBytes\s*\(|\.\s*transferTo\s*\(", "InputStream.readAllBytes / readNBytes / transferTo", 9),
    (r"\bFiles\s*\.\s*(readString|writeString)\s*\(|\bPath\s*\.\s*of\s*\(", "Files.readString / Path.of", 11),
    (r"\bObjects\s*\.\s*(requireNonNullElse|requireNonNullElseGet|checkIndex|checkFromToIndex|checkFromIndexSize)\s*\(",
     "Objects.requireNonNullElse / checkIndex", 9),
    (r"\bCollectors\s*\.\s*(toUnmodifiable\w*|teeing|filtering|flatMapping)\s*\(", "newer Collectors", 9),
    (r"\.\s*toList\s*\(\s*\)", "Stream.toList()", 16),
    (r"\.\s*(takeWhile|dropWhile)\s*\(", "Stream.takeWhile / dropWhile", 9),
    (r"\bPredicate\s*\.\s*not\s*\(", "Predicate.not", 11),
    (r"\bArrays\s*\.\s*(mismatch|compare)\s*\(", "Arrays.mismatch / compare", 9),
    (r"\bThread\s*\.\s*onSpinWait\s*\(|\bRuntime\s*\.\s*version\s*\(|\bProcessHandle\b|\bStackWalker\b", "Java 9 runtime APIs", 9),
    (r"\bVarHandle\b|\bjava\.util\.concurrent\.Flow\b|\bjava\.net\.http\b|\bjava\.lang\.foreign\b", "Java 9+ packages", 9),
    (r"\.\s*(orTimeout|completeOnTimeout)\s*\(", "CompletableFuture timeouts", 9),
    (r"\.\s*(position|limit|flip|clear|mark|reset|rewind)\s*\([^()]*\)\s*\.\s*(get\w*|put\w*|order|slice|duplicate|limit|position|flip|array)\b",
     "chained Buffer methods (covariant ByteBuffer returns: NoSuchMethodError on a Java 8 runtime)", 9),
    (r"(^|[;{}\s])(record|sealed|non-sealed|permits)\s+[A-Z]\w*", "records / sealed classes", 16),
    (r"\binstanceof\s+[\w.<>?,\s]+?\s+[a-z]\w*\s*[)&|;]", "pattern matching instanceof", 16),
    (r"case\s+[^:]*->", "switch expressions", 14),
    (r"\byield\s+[^;]+;", "switch yield", 14),
    (r"@Deprecated\s*\(\s*(since|forRemoval)", "@Deprecated(since / forRemoval)", 9),
    (r"\bmodule\s+[\w.]+\s*\{|\brequires\s+(transitive\s+)?[\w.]+\s*;", "module declarations", 9),
]


def strip_java(src: str) -> str:
    """The source with comments, string / char literals and text blocks blanked
    (line structure kept, so hits keep their line numbers)."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith('"""', i):
            j = src.find('"""', i + 3)
            j = n if j < 0 else j + 3
            out.append("\"\"\"TEXTBLOCK\"\"\"" + "\n" * src.count("\n", i, j))
            i = j
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("\n" * src.count("\n", i, j))
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c and src[j] != "\n":
                j += 2 if src[j] == "\\" else 1
            out.append(c + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def scan(src: str):
    code = strip_java(src)
    hits = []
    for ln, line in enumerate(code.split("\n"), 1):
        for pat, what, ver in POST_JAVA8:
            if re.search(pat, line):
                hits.append((ln, what, ver, line.strip()))
    if '"""TEXTBLOCK"""' in code:
        hits.append((0, "text blocks", 15, ""))
    return hits


def java_files():
    fs = []
    for d, _, names in os.walk(JAVA):
        fs += [os.path.join(d, f) for f in names if f.endswith(".java")]
    return sorted(fs)


@pytest.mark.skipif(not os.path.isdir(JAVA), reason="java/ not in this tree")
def test_drop_in_uses_nothing_newer_than_java8():
    files = java_files()
    assert len(files) >= 5, files
    bad = []
    for f in files:
        for ln, what, ver, line in scan(open(f, encoding="utf-8").read()):
            bad.append(f"{os.path.relpath(f, ROOT)}:{ln}: {what} (Java {ver}): {line}")
    assert not bad, "post-Java-8 API in the drop-in:\n" + "\n".join(bad)


@pytest.mark.skipif(not os.path.isdir(JAVA), reason="java/ not in this tree")
def test_event_release_is_java8():
    """The two event owners release through GpuRWI.EventHandle (a PhantomReference
    reaped by GpuRWI's thread), not java.lang.ref.Cleaner."""
    rwi = open(os.path.join(JAVA, "net/yacy/kelondro/rwi/GpuRWI.java")).read()
    assert "extends PhantomReference<Object>" in rwi and "ReferenceQueue" in rwi
    for rel in ("net/yacy/search/ranking/GpuReferenceOrder.java", "net/yacy/search/query/GpuRWIStack.java"):
        s = strip_java(open(os.path.join(JAVA, rel)).read())
        assert "gpu.track(this, this.event)" in s and "Cleaner" not in s, rel


@pytest.mark.parametrize("snippet", [
    "import java.lang.ref.Cleaner;",
    "private static final Cleaner C = Cleaner.create();",
    "final List<String> l = List.of(\"a\");",
    "var rows = new byte[40];",
    "for (var e : m.entrySet()) {}",
    "x = o.orElseThrow();",
    "if (s.isBlank()) return;",
    "t = s.strip();",
    "t = \"-\".repeat(3);",
    "byte[] b = in.readAllBytes();",
    "String s = Files.readString(p);",
    "List<Integer> l = st.toList();",
    "b.position(4).getLong();",
    "if (o instanceof Entry e) return e.score();",
    "int k = switch (x) { case 1 -> 2; default -> 3; };",
    "String t = \"\"\"\n  block\n  \"\"\";",
    "record Hit(long score) {}",
    "@Deprecated(since = \"9\")",
])
def test_scanner_catches(snippet):
    assert scan(snippet), snippet


@pytest.mark.parametrize("snippet", [
    "// java.lang.ref.Cleaner does the same from Java 9 on",
    "/* var x = List.of(1); */",
    "final String s = \"List.of(x) var y = 1\";",
    "final ByteBuffer b = ByteBuffer.wrap(hits).order(ByteOrder.LITTLE_ENDIAN);",
    "final long v = b.getLong(24 * h + 16);",
    "if (t instanceof Entry) return ((Entry) t).score();",
    "final Set<EventHandle> handles = Collections.newSetFromMap(new ConcurrentHashMap<EventHandle, Boolean>());",
    "for (final EventHandle h : new ArrayList<EventHandle>(this.handles)) h.release();",
    "final Reference<?> r = q.remove();",
    "int variance = 0; varName = 1;",
    "final java.util.stream.Stream<String> s = r.lines();",
    "switch (x) { case 1: y = 2; break; }",
])
def test_scanner_passes_java8(snippet):
    assert not scan(snippet), scan(snippet)
