{-# LANGUAGE ForeignFunctionInterface #-}
-- | Haskell binding of the MI355X batched Paxos engine (include/paxos_batch.h).
--
-- This is the module a maintainer adds next to the reference's src/Common.hs so
-- that app/Main.hs (/root/reference/app/Main.hs:27-53) can run batches of the
-- same single-decree protocol on GPUs instead of spawning Cloud Haskell
-- processes.  Results come back in the reference's vocabulary: 'Ticket'
-- (Common.hs:20-22), 'Command' = "c<clientId>.<t>" (Client.hs:202-203) and
-- 'Proposal' (Common.hs:29-30).
--
-- UNVERIFIED: neither this image nor the GPU box has GHC/stack/cabal
-- (SURVEY.md §8c), so this file has not been compiled.  The C side it binds is
-- exercised by tests/test_abi.py (symbols, struct layout) and the GPU tests.
--
-- The calls are `safe`: a batch blocks for the whole GPU run, and with the
-- threaded RTS (package.yaml:41-43, -threaded -with-rtsopts=-N) other
-- capabilities keep running meanwhile.
module PaxosBatch
  ( BatchConfig (..)
  , logConfig
  , Outcome (..)
  , Flag (..)
  , Totals (..)
  , defaultConfig
  , config2
  , runBatch
  , runBatchMulti
  , commandOf
    -- * Lifecycle (the host owns it: app/Main.hs start and exit)
  , abiVersion
  , initDevices
  , shutdown
  , withEngine
  , handoffCounts
    -- * Per-instance trace (the reference's `say` dumps, Server.hs:85, Client.hs:108)
  , AcceptorState (..)
  , ProposerState (..)
  , TraceStep (..)
  , traceInstance
  ) where

import           Common                (Command, Proposal, Ticket (..))

import           Control.Exception     (bracket_)
import           Control.Monad         (forM)
import           Data.Bits             (shiftR, testBit, (.&.))
import           Data.Int              (Int32, Int64)
import           Data.Word             (Word32, Word64)
import           Foreign.C.String      (CString, peekCString)
import           Foreign.C.Types       (CInt (..))
import           Foreign.ForeignPtr    (mallocForeignPtrArray, withForeignPtr)
import           Foreign.Marshal.Array (advancePtr, allocaArray, peekArray)
import           Foreign.Marshal.Utils (with)
import           Foreign.Ptr           (Ptr, nullPtr)
import           Foreign.Storable      (Storable (..))

-- | pxb_config (72 bytes, unchanged since ABI 3, see include/paxos_batch.h).
data BatchConfig = BatchConfig
  { bcSeed          :: !Word64
  , bcFirst         :: !Word64   -- ^ global id of the first instance
  , bcCount         :: !Word64   -- ^ instances in this batch
  , bcProposers     :: !Word32   -- ^ P, clientIds 1..P  (Main.hs:45 uses 2)
  , bcAcceptors     :: !Word32   -- ^ N                  (Main.hs:41 uses 2)
  , bcLossPpm       :: !Word32
  , bcDelayMax      :: !Word32
  , bcCrashPpm      :: !Word32
  , bcCrashLenMax   :: !Word32
  , bcCrashStartMax :: !Word32
  , bcSkewMax       :: !Word32
  , bcStepCap       :: !Word32
  , bcFlags         :: !Word32
  , bcTicks         :: !Word32   -- ^ log mode: Ticks per proposer (<= 1: single decree);
                                 --   the reference ticks forever (Client.hs:96-100)
  , bcTickPeriod    :: !Word32   -- ^ steps between Ticks
  } deriving (Show)

instance Storable BatchConfig where
  sizeOf _ = 72
  alignment _ = 8
  peek p = BatchConfig
    <$> peekByteOff p 0  <*> peekByteOff p 8  <*> peekByteOff p 16
    <*> peekByteOff p 24 <*> peekByteOff p 28 <*> peekByteOff p 32
    <*> peekByteOff p 36 <*> peekByteOff p 40 <*> peekByteOff p 44
    <*> peekByteOff p 48 <*> peekByteOff p 52 <*> peekByteOff p 56
    <*> peekByteOff p 60 <*> peekByteOff p 64 <*> peekByteOff p 68
  poke p c = do
    pokeByteOff p 0  (bcSeed c);        pokeByteOff p 8  (bcFirst c)
    pokeByteOff p 16 (bcCount c);       pokeByteOff p 24 (bcProposers c)
    pokeByteOff p 28 (bcAcceptors c);   pokeByteOff p 32 (bcLossPpm c)
    pokeByteOff p 36 (bcDelayMax c);    pokeByteOff p 40 (bcCrashPpm c)
    pokeByteOff p 44 (bcCrashLenMax c); pokeByteOff p 48 (bcCrashStartMax c)
    pokeByteOff p 52 (bcSkewMax c);     pokeByteOff p 56 (bcStepCap c)
    pokeByteOff p 60 (bcFlags c);       pokeByteOff p 64 (bcTicks c)
    pokeByteOff p 68 (bcTickPeriod c)

-- | The stock topology of app/Main.hs (2 acceptors, 2 proposers), fault-free.
defaultConfig :: BatchConfig
defaultConfig = BatchConfig 0x5EED0001 0 1 2 2 0 1 0 1 0 0 256 0 1 1

-- | The stock app/Main.hs run as the reference does it: both clients keep
-- ticking (here 16 Ticks, 8 steps apart), so the acceptor logs grow.
logConfig :: BatchConfig
logConfig = defaultConfig { bcTicks = 16, bcTickPeriod = 8, bcStepCap = 1024 }

-- | BASELINE config 2: 2^20 instances, 1 proposer, 5 acceptors, no faults.
config2 :: BatchConfig
config2 = defaultConfig { bcSeed = 0x5EED0002, bcCount = 2 ^ (20 :: Int)
                        , bcProposers = 1, bcAcceptors = 5 }

data Flag = Undecided | Stuck | Panic | LogDivergence | StepCap
          | QueueOverflow | TicketOverflow | LogTrunc
  deriving (Show, Eq, Enum, Bounded)

-- | One instance's outcome (pxb_result): the Proposal of the first Execute
-- broadcast (Client.hs:178), the number of AskForTicket rounds, the steps the
-- instance ran and its flags.
data Outcome = Outcome
  { oDecided :: Maybe Proposal
  , oRounds  :: !Int
  , oSteps   :: !Int
  , oFlags   :: [Flag]
  } deriving (Show)

-- | Run totals (pxb_counters, slots of SURVEY.md §8(e)).
data Totals = Totals
  { tDecided, tUndecided, tStuck, tPanic, tDivergence, tStepCap
  , tRounds, tMessages
  , tExecutes :: !Int64           -- ^ Execute broadcasts: commands committed (log mode)
  } deriving (Show)

-- | "c<clientId>.<t>" from the command code (Client.hs:202-203).
commandOf :: Word32 -> Command
commandOf code = "c" <> show (code `shiftR` 24) <> "." <> show (code .&. 0xFFFFFF)

foreign import ccall safe "pxb_run"
  c_pxb_run :: Ptr BatchConfig -> Ptr Word32 -> Ptr Word32 -> Ptr () -> Ptr Int64 -> IO CInt
foreign import ccall safe "pxb_run_multi"
  c_pxb_run_multi :: Ptr BatchConfig -> CInt -> Ptr Word32 -> Ptr Word32 -> Ptr () -> Ptr Int64 -> IO CInt
foreign import ccall unsafe "pxb_strerror"
  c_pxb_strerror :: CInt -> IO CString
foreign import ccall unsafe "pxb_abi_version"
  c_pxb_abi_version :: IO CInt
foreign import ccall safe "pxb_init"
  c_pxb_init :: CInt -> IO CInt
foreign import ccall safe "pxb_shutdown"
  c_pxb_shutdown :: IO CInt
foreign import ccall safe "pxb_handoff_counts"
  c_pxb_handoff_counts :: CInt -> Ptr Word64 -> CInt -> IO CInt
foreign import ccall safe "pxb_trace_instance"
  c_pxb_trace_instance :: Ptr BatchConfig -> Word64 -> Ptr Word32 -> Word32 -> Ptr Word32 -> Ptr Word32 -> IO CInt

-- | The ABI this module was written against (include/paxos_batch.h).
expectedAbi :: Int
expectedAbi = 5

-- | pxb_abi_version of the loaded library.
abiVersion :: IO Int
abiVersion = fromIntegral <$> c_pxb_abi_version

checked :: IO CInt -> IO (Either String ())
checked act = do
  rc <- act
  if rc == 0 then pure (Right ()) else Left <$> (c_pxb_strerror rc >>= peekCString)

-- | pxb_init: allocate the scratch of the first @g@ GPUs (all visible when
-- @g <= 0@) up front, at process start (where app/Main.hs:27-36 brings the
-- node up).  Optional: the first batch does it lazily.  Refuses a library
-- built for another ABI.
initDevices :: Int -> IO (Either String ())
initDevices g = do
  v <- abiVersion
  if v /= expectedAbi
    then pure (Left ("libpaxos_batch ABI " <> show v <> ", binding expects " <> show expectedAbi))
    else checked (c_pxb_init (fromIntegral g))

-- | pxb_shutdown: wait for the devices, free every scratch buffer and the
-- cached RCCL communicators (process exit).  No batch may be running on
-- another Haskell thread.
shutdown :: IO (Either String ())
shutdown = checked c_pxb_shutdown

-- | Bracket a program's batches with 'initDevices' / 'shutdown', so the
-- engine's lifetime is the host's, as the reference's node is
-- (app/Main.hs:27-53).
withEngine :: Int -> IO a -> IO (Either String a)
withEngine g body = do
  ok <- initDevices g
  case ok of
    Left err -> pure (Left err)
    Right () -> Right <$> bracket_ (pure ()) (shutdown >>= either putStrLn pure) body

-- | pxb_handoff_counts of GPU @dev@: instances the first per-lane kernel of a
-- chunk handed on, and those a second one handed on (observability only).
handoffCounts :: Int -> Bool -> IO (Either String (Word64, Word64))
handoffCounts dev reset =
  allocaArray 2 $ \p -> do
    r <- checked (c_pxb_handoff_counts (fromIntegral dev) p (if reset then 1 else 0))
    case r of
      Left err -> pure (Left err)
      Right () -> do
        [a, b] <- peekArray 2 p
        pure (Right (a, b))

-- | Run a batch on the current GPU.
runBatch :: BatchConfig -> IO (Either String ([Outcome], Totals))
runBatch cfg = runWith cfg (\pc pres ptot -> c_pxb_run pc pres nullPtr nullPtr ptot)

-- | Run a batch sharded over the first @g@ GPUs (all visible when @g <= 0@);
-- totals are all-reduced with RCCL.  Outcomes are identical to 'runBatch'.
runBatchMulti :: Int -> BatchConfig -> IO (Either String ([Outcome], Totals))
runBatchMulti g cfg =
  runWith cfg (\pc pres ptot -> c_pxb_run_multi pc (fromIntegral g) pres nullPtr nullPtr ptot)

runWith :: BatchConfig
        -> (Ptr BatchConfig -> Ptr Word32 -> Ptr Int64 -> IO CInt)
        -> IO (Either String ([Outcome], Totals))
runWith cfg call = do
  let n = fromIntegral (bcCount cfg) :: Int
  fres <- mallocForeignPtrArray (4 * n)          -- pinned: 16 B per instance
  with cfg $ \pc ->
    withForeignPtr fres $ \pres ->
      allocaArray 16 $ \ptot -> do
        rc <- call pc pres ptot
        if rc /= 0
          then Left <$> (c_pxb_strerror rc >>= peekCString)
          else do
            outs <- forM [0 .. n - 1] $ \i -> do
              [v, t, r, f] <- peekArray 4 (advancePtr pres (4 * i))
              pure (decode v t r f)
            tot <- peekArray 16 ptot
            let [d, u, s, p, dv, sc, rd, ms] = take 8 tot
            pure (Right (outs, Totals d u s p dv sc rd ms (tot !! 14)))

decode :: Word32 -> Word32 -> Word32 -> Word32 -> Outcome
decode v t r f = Outcome
  { oDecided = if v == 0 then Nothing
               else Just (Ticket (fromIntegral (fromIntegral t :: Int32)), commandOf v)
  , oRounds  = fromIntegral r
  , oSteps   = fromIntegral (f `shiftR` 16)
  , oFlags   = [fl | fl <- [minBound .. maxBound], testBit f (fromEnum fl)]
  }

-- | An acceptor at the end of a traced step (ServerState, Server.hs:24-31).
data AcceptorState = AcceptorState
  { asLargestTicket :: Ticket
  , asProposal      :: Maybe Proposal
  , asLogLength     :: !Int
  , asDead          :: !Bool         -- ^ after a Server.hs:76 panic (Q6)
  , asLogDigest     :: !Word32       -- ^ FNV-1a of its log so far (docs/SEMANTICS.md §7)
  } deriving (Show)

-- | A proposer at the end of a traced step (ClientState, Client.hs:58-67).
data ProposerState = ProposerState
  { psTicket     :: Ticket
  , psCommand    :: Maybe Command    -- ^ _mCommand
  , psAcks       :: !Int
  , psPhase      :: !Int             -- ^ 0 Idle, 1 Round1, 2 Round2
  , psMostRecent :: Maybe Proposal   -- ^ Round1: MostRecent
  , psRound2     :: Maybe Command    -- ^ Round2: the proposed command
  , psPending    :: !Bool            -- ^ Round2: _originalCommandPending
  } deriving (Show)

-- | One record of 'traceInstance': the state after a step (steps with nothing
-- due and no Tick change nothing and are skipped).  'tsInFlight' is Nothing
-- when copies of a broadcast were still to be sent (production variant only).
data TraceStep = TraceStep
  { tsStep      :: !Int
  , tsInFlight  :: Maybe Int
  , tsAcceptors :: [AcceptorState]
  , tsProposers :: [ProposerState]
  } deriving (Show)

-- | pxb_trace_instance: instance @i@ of @cfg@ (single decree or, ABI 5, log
-- mode) on one GPU lane, its state recorded at the end of every step, at most
-- @maxRecords@ records; with its outcome.  What 'runBatch' cannot show: where
-- a run departs from the reference's schedule, step by step.
traceInstance :: BatchConfig -> Word64 -> Int -> IO (Either String ([TraceStep], Outcome))
traceInstance cfg i maxRecords = do
  let nw = 73                                      -- sizeof(pxb_trace_step) / 4
  buf <- mallocForeignPtrArray (nw * maxRecords)
  with cfg { bcFirst = i, bcCount = 1 } $ \pc ->
    withForeignPtr buf $ \pb ->
      allocaArray 1 $ \pn ->
        allocaArray 4 $ \pres -> do
          rc <- c_pxb_trace_instance pc i pb (fromIntegral maxRecords) pn pres
          if rc /= 0
            then Left <$> (c_pxb_strerror rc >>= peekCString)
            else do
              [n] <- peekArray 1 pn
              recs <- forM [0 .. fromIntegral n - 1] $ \k -> step <$> peekArray nw (advancePtr pb (nw * k))
              [v, t, r, f] <- peekArray 4 pres
              pure (Right (recs, decode v t r f))
  where
    step w =
      let at k = w !! k
          nA = fromIntegral (at 2); nP = fromIntegral (at 3)
          cmd c = if c == 0 then Nothing else Just (commandOf c)
          prop t c = if c == 0 then Nothing else Just (Ticket (fromIntegral (fromIntegral t :: Int32)), commandOf c)
          acc a = let b = 4 + 4 * a; meta = at (b + 3)
                  in AcceptorState (Ticket (fromIntegral (fromIntegral (at b) :: Int32))) (prop (at (b + 1)) (at (b + 2)))
                                   (fromIntegral (meta .&. 0x7FFFFFFF)) (testBit meta 31) (at (40 + a))
          pro q = let b = 49 + 8 * q
                  in ProposerState (Ticket (fromIntegral (fromIntegral (at b) :: Int32))) (cmd (at (b + 1)))
                                   (fromIntegral (at (b + 2))) (fromIntegral (at (b + 3))) (prop (at (b + 4)) (at (b + 5)))
                                   (cmd (at (b + 6))) (at (b + 7) /= 0)
      in TraceStep (fromIntegral (at 0)) (if at 1 == 0xFFFFFFFF then Nothing else Just (fromIntegral (at 1)))
                   (map acc [0 .. nA - 1]) (map pro [0 .. nP - 1])
