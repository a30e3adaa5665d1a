-- | Batch driver replacing the actor-spawning body of app/Main.hs
-- (/root/reference/app/Main.hs:27-53): instead of one Cloud Haskell node with
-- 2 servers and 2 clients logging forever, run BASELINE config 2 (or the
-- stock 2x2 topology) as a GPU batch through the C ABI and print the outcome
-- in the reference's vocabulary.  UNVERIFIED (no GHC in this image).
module Main where

import           PaxosBatch

import           System.Environment (getArgs)

main :: IO ()
main = do
  args <- getArgs
  let cfg = case args of
        ["stock"] -> defaultConfig { bcCount = 1 }   -- Main.hs:41,45: 2 servers, 2 clients
        _         -> config2
  -- the engine lives as long as this process (pxb_init at start, pxb_shutdown at exit)
  e <- withEngine 0 $ do
    r <- runBatchMulti 0 cfg
    case r of
      Left err -> putStrLn ("pxb error: " ++ err)
      Right (outs, tot) -> do
        print tot
        mapM_ print (take 4 outs)
  either (putStrLn . ("pxb init: " ++)) pure e
