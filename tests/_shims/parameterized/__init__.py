"""Tiny stand-in for the ``parameterized`` package (absent from this image, no network).

Only ``parameterized.expand`` is provided — the one entry point the reference's unittest suite
uses — so the reference tests can run against this framework unchanged.
"""
import functools


class parameterized:  # noqa: N801 - mirror the real package's API
    @staticmethod
    def expand(cases):
        def decorate(fn):
            import inspect
            frame = inspect.currentframe().f_back
            for i, case in enumerate(cases):
                args = case if isinstance(case, (tuple, list)) else (case,)

                def make(args=args):
                    @functools.wraps(fn)
                    def test(self):
                        return fn(self, *args)
                    return test
                frame.f_locals[f"{fn.__name__}_{i}"] = make()
            return None
        return decorate
