"""CPU checks of LDS layouts against the gfx950 bank rules
(MI355X_MICROARCH.md §LDS): the large-batch weight-gradient kernel's image
(iwae_dwgrad.hip) -- transposed fragment reads and row-major staging writes --
has no bank conflicts."""
import os
import runpy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dw_image_is_conflict_free(capsys):
    runpy.run_path(os.path.join(ROOT, "tools", "dw_banks.py"), run_name="__main__")
    out = capsys.readouterr().out
    assert "tr read worst way 1" in out
    assert "write worst way 1" in out
