"""`python -m ndfl.gzip InputFile OutputFile.gz` -- S/gzip.java over the GPU codec (see ndfl.cli)."""
from .cli import _main, gzip_submain

if __name__ == "__main__":
    _main(gzip_submain)
