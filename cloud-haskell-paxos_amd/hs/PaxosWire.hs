{-# LANGUAGE ForeignFunctionInterface #-}
-- | Haskell binding of the GPU wire codec (include/paxos_batch.h, pxb_wire_*).
--
-- Batch form of the bytes that `send` puts on the wire for `contentOf m` in
-- sendMessages (/root/reference/src/Common.hs:36-39).  Those bytes come from the
-- generic 'Binary' instances of 'ClientRequest' and 'ServerResponse'
-- (Common.hs:41-55), and 'encodeRequests' / 'encodeResponses' produce exactly
-- what 'Data.Binary.encode' of each value does (oracle/wire_ref.py restates it;
-- tests/test_wire.py checks the GPU against it).  Cloud Haskell's envelope
-- (the sender ProcessId of the tuple, the type fingerprint, the transport
-- framing) stays with the node.
--
-- UNVERIFIED: no GHC in this image or on the GPU box (SURVEY.md §8c); this file
-- has not been compiled.  The C entry points are covered by tests/test_abi.py
-- and tests/test_wire.py.
module PaxosWire
  ( encodeRequests
  , encodeResponses
  , decodeRequests
  , decodeResponses
  , WireError (..)
  , codeOf
  ) where

import           Common                   (ClientRequest (..), Command, ServerResponse (..), Ticket (..))
import           PaxosBatch               (commandOf)

import qualified Data.ByteString          as BS
import qualified Data.ByteString.Unsafe   as BSU
import           Data.Bits                (shiftL, (.|.))
import           Data.Char                (isDigit)
import           Data.Int                 (Int32)
import           Data.Word                (Word32, Word64, Word8)
import           Foreign.C.Types          (CInt (..))
import           Foreign.Marshal.Alloc    (alloca)
import           Foreign.Marshal.Array    (allocaArray, peekArray, pokeArray, withArray)
import           Foreign.Ptr              (Ptr, castPtr)
import           Foreign.Storable         (peek)

-- | Per-record decode status (PXB_WIRE_E_*).
data WireError = WireLength | WireTag | WireString | WireRange | WireOther Word32
  deriving (Show, Eq)

foreign import ccall safe "pxb_wire_encode_host"
  c_encode :: Ptr Word32 -> Word64 -> Word32 -> Ptr Word8 -> Ptr Word64 -> Ptr Word64 -> IO CInt
foreign import ccall safe "pxb_wire_decode_host"
  c_decode :: Ptr Word8 -> Word64 -> Ptr Word64 -> Word64 -> Word32 -> Ptr Word32 -> Ptr Word32 -> IO CInt

wireRequest, wireResponse, maxBytes :: Word32
wireRequest = 0
wireResponse = 1
maxBytes = 39

-- | The command code (clientId << 24 | t) of "c<clientId>.<t>" (Client.hs:202-203).
codeOf :: Command -> Maybe Word32
codeOf ('c' : rest) = case break (== '.') rest of
  (i, '.' : t) | ok i, ok t, read i < (256 :: Integer), read t < (2 ^ (24 :: Int) :: Integer) ->
    Just ((read i `shiftL` 24) .|. read t)
  _ -> Nothing
  where ok s = not (null s) && all isDigit s && (s == "0" || head s /= '0')
codeOf _ = Nothing

-- pxb_msg words: kind, x, y, z
type Msg = (Word32, Int32, Int32, Word32)

ticket :: Ticket -> Int32
ticket (Ticket t) = fromIntegral t

reqMsg :: ClientRequest -> Maybe Msg
reqMsg (AskForTicket t)   = Just (0, ticket t, 0, 0)
reqMsg (Propose (t, c))   = (\z -> (1, ticket t, 0, z)) <$> codeOf c
reqMsg (Execute t)        = Just (2, ticket t, 0, 0)

respMsg :: ServerResponse -> Maybe Msg
respMsg (Round1OK t Nothing)        = Just (0, ticket t, 0, 0)
respMsg (Round1OK t (Just (s, c)))  = (\z -> (0, ticket t, ticket s, z)) <$> codeOf c
respMsg (HaveTicket t)              = Just (1, ticket t, 0, 0)
respMsg Round2Success               = Just (2, 0, 0, 0)

-- | Data.Binary bytes of every request, concatenated, with the n + 1 offsets.
-- Nothing when a command is not a "c<id>.<t>" the engine can carry.
encodeRequests :: [ClientRequest] -> IO (Either String (BS.ByteString, [Word64]))
encodeRequests = encodeWith wireRequest . traverse reqMsg

encodeResponses :: [ServerResponse] -> IO (Either String (BS.ByteString, [Word64]))
encodeResponses = encodeWith wireResponse . traverse respMsg

encodeWith :: Word32 -> Maybe [Msg] -> IO (Either String (BS.ByteString, [Word64]))
encodeWith _ Nothing = pure (Left "command outside the engine's \"c<id>.<t>\" range")
encodeWith ty (Just ms) = do
  let n = length ms
      words32 = concat [[k, fromIntegral x, fromIntegral y, z] | (k, x, y, z) <- ms]
  withArray words32 $ \pm ->
    allocaArray (max 1 (n * fromIntegral maxBytes)) $ \pout ->
      allocaArray (n + 1) $ \poffs ->
        alloca $ \pnb -> do
          rc <- c_encode pm (fromIntegral n) ty pout poffs pnb
          if rc /= 0
            then pure (Left ("pxb_wire_encode_host failed: " <> show rc))
            else do
              nb <- peek pnb
              bytes <- BS.packCStringLen (castPtr pout, fromIntegral nb)
              offs <- peekArray (n + 1) poffs
              pure (Right (bytes, offs))

-- | Decode records framed by @offsets@ (n + 1 entries): per record the value
-- or its 'WireError', as `Data.Binary.decodeOrFail` would accept or reject it.
decodeRequests :: BS.ByteString -> [Word64] -> IO (Either String [Either WireError ClientRequest])
decodeRequests = decodeWith wireRequest toReq
  where toReq (0, x, _, _) = AskForTicket (tk x)
        toReq (1, x, _, z) = Propose (tk x, commandOf z)
        toReq (_, x, _, _) = Execute (tk x)

decodeResponses :: BS.ByteString -> [Word64] -> IO (Either String [Either WireError ServerResponse])
decodeResponses = decodeWith wireResponse toResp
  where toResp (0, x, _, 0) = Round1OK (tk x) Nothing
        toResp (0, x, y, z) = Round1OK (tk x) (Just (tk y, commandOf z))
        toResp (1, x, _, _) = HaveTicket (tk x)
        toResp _            = Round2Success

tk :: Int32 -> Ticket
tk = Ticket . fromIntegral

decodeWith :: Word32 -> (Msg -> a) -> BS.ByteString -> [Word64] -> IO (Either String [Either WireError a])
decodeWith ty conv bytes offsets = do
  let n = length offsets - 1
  if n <= 0 then pure (Right []) else
    BSU.unsafeUseAsCString (if BS.null bytes then BS.singleton 0 else bytes) $ \pin ->
      withArray offsets $ \poffs ->
        allocaArray (4 * n) $ \pm ->
          allocaArray n $ \pst -> do
            pokeArray pst (replicate n 0)
            rc <- c_decode (castPtr pin) (fromIntegral (BS.length bytes)) poffs (fromIntegral n) ty pm pst
            if rc /= 0
              then pure (Left ("pxb_wire_decode_host failed: " <> show rc))
              else do
                ws <- peekArray (4 * n) pm
                st <- peekArray n pst
                let msgs = chunk ws
                pure (Right (zipWith (\s m -> if s == 0 then Right (conv m) else Left (err s)) st msgs))
  where
    chunk (k : x : y : z : r) = (k, fromIntegral x, fromIntegral y, z) : chunk r
    chunk _ = []
    err 1 = WireLength
    err 2 = WireTag
    err 3 = WireString
    err 4 = WireRange
    err s = WireOther s
