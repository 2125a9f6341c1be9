from .SCDecoder import SCDecoder  # noqa: F401
from .SCLUTDecoder import SCLUTDecoder  # noqa: F401
from .SCLLUTDecoder import SCLLUTDecoder  # noqa: F401
from .FastSCLUTDecoder import FastSCLUTDecoder  # noqa: F401
from .FastSCLLUTDecoder import FastSCLLUTDecoder  # noqa: F401
