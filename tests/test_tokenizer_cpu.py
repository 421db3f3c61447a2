"""Native caption tokenizer (csrc/tokenizer, dalle_amd._tokenizer) against the Rust ``tokenizers`` library
and ``transformers.T5TokenizerFast`` -- the reference's tokenizer (reference task.py:58, data.py:24).

No T5 vocabulary is available offline, so the fixtures train small SentencePiece unigram models
locally (nmt_nfkc normalisation -> the same precompiled-charsmap pipeline t5-small ships) and convert
them with transformers' own slow->fast converter; parity on the real t5-small vocabulary is unpinned.
"""
import json
import os
import random
import shutil
import subprocess

import pytest

spm = pytest.importorskip("sentencepiece")
tokenizers = pytest.importorskip("tokenizers")
transformers = pytest.importorskip("transformers")

from dalle_amd.data.tokenizer import NativeUnigramTokenizer, UnsupportedPipeline, load_tokenizer  # noqa: E402

ALPHABET = (list("abcdefghijklmnopqrstuvwxyz ABCXYZ  ,.!?-()'\"0123456789") + list("éèüñçøåßæœ")
            + ["ﬁ", "①", "Ｆ", "ｕ", "\xa0", "\t", "\n", "é", "　", "😀", "👍🏽", "中文", "カタカナ", "ｶﾀｶﾅ",
               "</s>", "<pad>", "<extra_id_5>", "  ", "™", "½", "Ⅻ", "​", "‍", "\r\n"])


def _corpus(path, lines=6000, seed=0):
    rng = random.Random(seed)
    syl = ["ka", "ro", "mi", "te", "su", "na", "lo", "pe", "qui", "dra", "ston", "ble", "ing", "tion", "er", "al"]
    base = ("a red apple on the table photo of cat dog sitting near blue sky painting by van gogh city night "
            "café naïve übermensch Ｆｕｌｌ ﬁne ① , . ! ? - ( ) 2021").split()
    words = base + ["".join(rng.choice(syl) for _ in range(rng.randint(1, 4))) for _ in range(1500)]
    with open(path, "w", encoding="utf-8") as f:
        for _ in range(lines):
            f.write(" ".join(rng.choice(words) for _ in range(rng.randint(3, 12))) + "\n")


@pytest.fixture(scope="module")
def t5_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("t5tok")
    _corpus(d / "corpus.txt")
    spm.SentencePieceTrainer.train(input=str(d / "corpus.txt"), model_prefix=str(d / "spiece"), vocab_size=800,
                                   model_type="unigram", normalization_rule_name="nmt_nfkc", pad_id=0, eos_id=1,
                                   unk_id=2, bos_id=-1, minloglevel=2)
    from transformers import T5Tokenizer
    from transformers.convert_slow_tokenizer import convert_slow_tokenizer

    slow = T5Tokenizer(vocab_file=str(d / "spiece.model"), extra_ids=100)
    convert_slow_tokenizer(slow).save(str(d / "tokenizer.json"))
    return d


def _cases(n, seed=1):
    rng = random.Random(seed)
    out = ["a red  apple, Café!! zzz  ﬁne ① </s>x", "", " ", "   lead and trail   ", "ＡＢＣ full width", "naïve übermensch"]
    out += ["".join(rng.choice(ALPHABET) for _ in range(rng.randint(0, 40))) for _ in range(n)]
    return out


def test_native_matches_tokenizers_library(t5_dir):
    tj = str(t5_dir / "tokenizer.json")
    assert json.load(open(tj))["normalizer"] is not None  # the precompiled charsmap path is exercised
    nat = NativeUnigramTokenizer(tj)
    lib = tokenizers.Tokenizer.from_file(tj)
    cases = _cases(2000)
    got = nat(cases, add_special_tokens=False)["input_ids"]
    for c, ids in zip(cases, got):
        assert ids == lib.encode(c, add_special_tokens=False).ids, repr(c)
    with_eos = nat(cases[:300], add_special_tokens=True)["input_ids"]
    for c, ids in zip(cases, with_eos):
        assert ids == lib.encode(c).ids, repr(c)


def test_native_matches_transformers_call_semantics(t5_dir):
    """``tokenizer(texts, add_special_tokens=..., max_length=..., truncation=True)`` as the reference calls
    it, through transformers' fast-tokenizer wrapper over the same file (the version-dependent T5
    'legacy' prefix rewriting of newer transformers releases is not part of the reference's pipeline)."""
    from transformers import PreTrainedTokenizerFast

    hf = PreTrainedTokenizerFast(tokenizer_file=str(t5_dir / "tokenizer.json"), eos_token="</s>", pad_token="</s>",
                                 unk_token="<unk>")
    nat = load_tokenizer(str(t5_dir))
    assert isinstance(nat, NativeUnigramTokenizer)
    assert nat.vocab_size == len(hf) and nat.eos_token_id == nat.pad_token_id == 1 and nat.unk_token_id == 2
    cases = _cases(200, seed=7)
    for special in (False, True):
        for ml in (1, 3, 8, 256):
            a = nat(cases, add_special_tokens=special, max_length=ml, truncation=True)
            b = hf(cases, add_special_tokens=special, max_length=ml, truncation=True)
            assert a["input_ids"] == b["input_ids"], (special, ml)
            assert a["attention_mask"] == b["attention_mask"]
    single = nat("a red apple", add_special_tokens=False, max_length=256, truncation=True)
    assert single["input_ids"] == hf("a red apple", add_special_tokens=False)["input_ids"]


def test_python_unicode_prefix_and_regex_replace():
    """NFKC (applied in Python before the native steps) + a regex Replace + WhitespaceSplit/Metaspace
    with the 'first' prepend scheme, trained with the tokenizers library itself."""
    from tokenizers import Regex, Tokenizer, models, normalizers, pre_tokenizers, processors, trainers

    rng = random.Random(3)
    words = "a red apple on the table photo café naïve Ｆｕｌｌ ﬁne ① cat dog".split()
    texts = [" ".join(rng.choice(words) for _ in range(rng.randint(2, 9))) for _ in range(2000)]
    tok = Tokenizer(models.Unigram())
    tok.normalizer = normalizers.Sequence([normalizers.NFKC(), normalizers.Replace(Regex(" {2,}"), " ")])
    tok.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.WhitespaceSplit(),
                                                 pre_tokenizers.Metaspace(prepend_scheme="first")])
    tok.train_from_iterator(texts, trainers.UnigramTrainer(vocab_size=120, special_tokens=["<pad>", "</s>", "<unk>"],
                                                           unk_token="<unk>"))
    tok.post_processor = processors.TemplateProcessing(single="$A </s>", special_tokens=[("</s>", 1)])
    import tempfile, os  # noqa: E401

    with tempfile.TemporaryDirectory() as d:
        tj = os.path.join(d, "tokenizer.json")
        tok.save(tj)
        nat = NativeUnigramTokenizer(tj)
    for c in _cases(1500, seed=11):
        assert nat(c, add_special_tokens=True)["input_ids"] == tok.encode(c).ids, repr(c)


def test_unsupported_pipeline_falls_back_to_library(tmp_path):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE(unk_token="<unk>"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.train_from_iterator(["a red apple on the table"] * 50, trainers.BpeTrainer(vocab_size=60, special_tokens=["<unk>"]))
    tok.save(str(tmp_path / "tokenizer.json"))
    with pytest.raises(UnsupportedPipeline):
        NativeUnigramTokenizer(str(tmp_path / "tokenizer.json"))
    fallback = load_tokenizer(str(tmp_path))
    assert not isinstance(fallback, NativeUnigramTokenizer)
    assert fallback("a red apple", add_special_tokens=False)["input_ids"] == tok.encode("a red apple").ids


SANITIZERS = {
    "tsan": ["-fsanitize=thread"],
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("kind", sorted(SANITIZERS))
def test_tokenizer_core_under_sanitizers(kind, t5_dir, tmp_path):
    """Random / invalid UTF-8 through the pybind-free core on 4 threads sharing one pipeline, under
    TSan and ASan+UBSan, with the trained model's vocabulary and precompiled charsmap."""
    import base64

    spec = json.load(open(t5_dir / "tokenizer.json"))
    with open(tmp_path / "vocab.tsv", "wb") as f:
        for piece, score in spec["model"]["vocab"]:
            f.write(piece.encode() + b"\t" + repr(float(score)).encode() + b"\n")
    norm = spec["normalizer"]
    steps = norm["normalizers"] if norm.get("type") == "Sequence" else [norm]
    blob = next(st["precompiled_charsmap"] for st in steps if st.get("type") == "Precompiled")
    (tmp_path / "charsmap.bin").write_bytes(base64.b64decode(blob))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "csrc", "tokenizer", "tokenizer_fuzz.cpp")
    exe = str(tmp_path / f"tokenizer_fuzz_{kind}")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *SANITIZERS[kind], "-I", os.path.dirname(src), src, "-o", exe,
                    "-pthread"], check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="halt_on_error=1 detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), "4", "3000"], capture_output=True, text=True, timeout=240, env=env)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "WARNING: ThreadSanitizer" not in report and "ERROR: AddressSanitizer" not in report, report[-4000:]
    assert "runtime error:" not in report, report[-4000:]
    assert "tokenizer fuzz ok" in r.stdout


def test_encode_batch_worker_errors_raise_in_python():
    """A worker thread's exception is re-raised on the calling thread as a Python exception (ADVICE r2:
    it used to std::terminate the data-loader process); an unconfigured pipeline raises instead of
    dereferencing an empty model."""
    import pytest

    tok = pytest.importorskip("dalle_amd._tokenizer")
    p = tok.Pipeline()
    with pytest.raises(RuntimeError, match="no model"):
        p.encode("abc")
    with pytest.raises(RuntimeError, match="no model"):
        p.encode_batch(["abc def"] * 200, threads=4)
