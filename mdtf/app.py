"""``tf.app.run`` analogue: parse flags, call ``main(argv)``, exit with its code."""
import sys

from .config.flags import FLAGS


def run(main=None, argv=None):
    rest = FLAGS(argv if argv is not None else sys.argv[1:])
    if main is None:
        main = sys.modules["__main__"].main
    code = main([sys.argv[0]] + list(rest))
    sys.exit(code if isinstance(code, int) else 0)
