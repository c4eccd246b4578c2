"""Every recipe script under tools/ is evidence for a measurement: each
tools/*.sh must be cited (by file name) in DESIGN.md or in a profiles/ file,
so that the directory holds no uncited one-off scripts."""
import glob
import os

from conftest import REPO


def _corpus():
    texts = []
    with open(os.path.join(REPO, 'DESIGN.md'), encoding='utf-8') as fh:
        texts.append(fh.read())
    for fn in glob.glob(os.path.join(REPO, 'profiles', '*')):
        if os.path.isfile(fn):
            with open(fn, encoding='utf-8', errors='replace') as fh:
                texts.append(fh.read())
    return '\n'.join(texts)


def test_every_tools_script_is_cited():
    corpus = _corpus()
    scripts = sorted(os.path.basename(p) for p in glob.glob(os.path.join(REPO, 'tools', '*.sh')))
    assert scripts
    uncited = [s for s in scripts if s not in corpus]
    assert not uncited, uncited
